#!/bin/bash
# Round-4 closing GPU session: smoke, the whole GPU suite, the driver's bench command, a two-rank torchrun
# rehearsal on the one GPU, the in-process path over 4 and 8 CU partitions (node time-to-work), and the
# receive-difficulty workload.  Every step has its own time limit; the chain stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r04f}
PYT="python3 -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 180 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 &&
timeout -k 10 900 $PYT tests -m gpu > gpurun_out/${T}_pytest_gpu.log 2>&1 &&
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err &&
timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 40 --warmup 3 --node-searches 100 > gpurun_out/${T}_torchrun2_shared_gpu.json 2> gpurun_out/${T}_torchrun2.err &&
NANOPOW_VIRTUAL_DEVICES=4 timeout -k 10 400 python3 bench.py --gpus 4 --steps 40 --warmup 3 --node-searches 300 > gpurun_out/${T}_inproc_4cu.json 2> gpurun_out/${T}_inproc_4cu.err &&
NANOPOW_VIRTUAL_DEVICES=8 timeout -k 10 400 python3 bench.py --gpus 8 --steps 40 --warmup 3 --node-searches 300 > gpurun_out/${T}_inproc_8cu.json 2> gpurun_out/${T}_inproc_8cu.err &&
timeout -k 10 400 python3 bench.py --workload receive --steps 300 > gpurun_out/${T}_receive.json 2> gpurun_out/${T}_receive.err
rc=$?
tail -n 2 gpurun_out/${T}_pytest_gpu.log; head -c 400 gpurun_out/${T}_bench.json; echo; head -c 300 gpurun_out/${T}_inproc_8cu.json
exit $rc
