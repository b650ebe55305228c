#!/bin/bash
# Round-3 closing GPU session: smoke, the whole GPU suite, the driver's bench command, a two-rank
# torchrun rehearsal on the one GPU (the box narrows ROCR_VISIBLE_DEVICES to it, so both ranks keep it) and the receive-difficulty workload.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r03f}
PYT="python3 -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 180 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 &&
timeout -k 10 900 $PYT tests -m gpu > gpurun_out/${T}_pytest_gpu.log 2>&1 &&
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err &&
timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 40 --warmup 3 --node-searches 100 > gpurun_out/${T}_torchrun2_shared_gpu.json 2> gpurun_out/${T}_torchrun2.err &&
timeout -k 10 400 python3 bench.py --workload receive --steps 300 > gpurun_out/${T}_receive.json 2> gpurun_out/${T}_receive.err
rc=$?
tail -2 gpurun_out/${T}_pytest_gpu.log; head -c 400 gpurun_out/${T}_bench.json; echo; head -c 400 gpurun_out/${T}_torchrun2_shared_gpu.json
exit $rc
