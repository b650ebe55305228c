#!/bin/bash
# Round-5 closing GPU session: smoke, the driver's bench command (no flags, and --steps 20 --warmup 5), a two-rank
# torchrun rehearsal on the one GPU, the in-process path over 4 and 8 CU partitions (lingering launches on there by
# default), the receive-difficulty workload, the 8-GPU time regime over 8 partitions and on the whole GPU.  Every step
# has its own time limit; the chain stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r05f}
timeout -k 10 180 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 &&
timeout -k 10 400 python3 bench.py > gpurun_out/${T}_bench_noflags.json 2> gpurun_out/${T}_bench_noflags.err &&
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err &&
timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 40 --warmup 3 --node-searches 100 > gpurun_out/${T}_torchrun2_shared_gpu.json 2> gpurun_out/${T}_torchrun2.err &&
NANOPOW_VIRTUAL_DEVICES=4 timeout -k 10 400 python3 bench.py --gpus 4 --steps 40 --warmup 3 --node-searches 300 > gpurun_out/${T}_inproc_4cu.json 2> gpurun_out/${T}_inproc_4cu.err &&
NANOPOW_VIRTUAL_DEVICES=8 timeout -k 10 400 python3 bench.py --gpus 8 --steps 40 --warmup 3 --node-searches 300 > gpurun_out/${T}_inproc_8cu.json 2> gpurun_out/${T}_inproc_8cu.err &&
timeout -k 10 400 python3 bench.py --workload receive --steps 300 > gpurun_out/${T}_receive.json 2> gpurun_out/${T}_receive.err &&
NANOPOW_VIRTUAL_DEVICES=8 timeout -k 10 400 python3 bench.py --workload regime --gpus 8 --steps 2000 --http-requests 200 > gpurun_out/${T}_regime8.json 2> gpurun_out/${T}_regime8.err &&
timeout -k 10 400 python3 bench.py --workload regime --gpus 1 --steps 2000 --http-requests 200 > gpurun_out/${T}_regime1.json 2> gpurun_out/${T}_regime1.err
rc=$?
head -c 600 gpurun_out/${T}_bench.json; echo; head -c 300 gpurun_out/${T}_inproc_8cu.json
exit $rc
