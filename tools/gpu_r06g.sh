#!/bin/bash
# Round-6 closing GPU session, part 2 (the final build's evidence): the profiling recipe (tools/prof_r06.sh: rocprofv3
# timed region with the regime child kept in, PMC passes of the search and sweep kernels, dual issue), then the 8-GPU
# time regime over 8 CU partitions and on the whole GPU, the receive workload, two torchrun ranks on the one GPU and
# the in-process path over 4 and 8 partitions.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r06f}
bash tools/prof_r06.sh $T > gpurun_out/${T}_prof.log 2>&1 &&
NANOPOW_VIRTUAL_DEVICES=8 timeout -k 10 400 python3 bench.py --workload regime --gpus 8 --steps 2000 --http-requests 200 > gpurun_out/${T}_regime8.json 2> gpurun_out/${T}_regime8.err &&
timeout -k 10 400 python3 bench.py --workload regime --gpus 1 --steps 2000 --http-requests 200 > gpurun_out/${T}_regime1.json 2> gpurun_out/${T}_regime1.err &&
timeout -k 10 400 python3 bench.py --workload receive --steps 300 > gpurun_out/${T}_receive.json 2> gpurun_out/${T}_receive.err &&
timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 40 --warmup 3 --node-searches 100 > gpurun_out/${T}_torchrun2_shared_gpu.json 2> gpurun_out/${T}_torchrun2.err &&
NANOPOW_VIRTUAL_DEVICES=4 timeout -k 10 400 python3 bench.py --gpus 4 --steps 40 --warmup 3 --node-searches 300 > gpurun_out/${T}_inproc_4cu.json 2> gpurun_out/${T}_inproc_4cu.err &&
NANOPOW_VIRTUAL_DEVICES=8 timeout -k 10 400 python3 bench.py --gpus 8 --steps 40 --warmup 3 --node-searches 300 > gpurun_out/${T}_inproc_8cu.json 2> gpurun_out/${T}_inproc_8cu.err
rc=$?
tail -30 gpurun_out/${T}_prof.log
for f in regime8 regime1 receive torchrun2_shared_gpu inproc_4cu inproc_8cu; do echo "$f"; head -c 300 gpurun_out/${T}_$f.json; echo; done
exit $rc
