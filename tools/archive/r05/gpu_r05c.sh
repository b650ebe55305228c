#!/bin/bash
# Round 5, session c: (1) the stop span against the number of CU partitions (2..8) -- is the 8-partition tail the
# hardware queues (8 CU-masked queues beside HIP's own) rather than the engine?; (2) the regime on the build with
# the win watcher, per-job waits and per-device wake-ups, watcher on / off; (3) the GPU suite; (4) A/B watcher on/off
# on the one-GPU bench workload.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r05c}
PYT="python3 -u -m pytest -x -v --timeout 300 --timeout-method thread"
R="python3 bench.py --workload regime --steps 1000 --http-requests 200"
for G in 2 3 4 5 6 7 8; do
  NANOPOW_TEST_HOOKS=1 NANOPOW_VIRTUAL_DEVICES=$G timeout -k 10 200 python3 tests/overshoot_worker.py 100 receive > gpurun_out/${T}_over_g$G.json 2> gpurun_out/${T}_over_g$G.err || exit $?
done
GPU_MAX_HW_QUEUES=1 NANOPOW_TEST_HOOKS=1 NANOPOW_VIRTUAL_DEVICES=8 timeout -k 10 200 python3 tests/overshoot_worker.py 100 receive > gpurun_out/${T}_over_g8_hwq1.json 2> gpurun_out/${T}_over_g8_hwq1.err &&
NANOPOW_VIRTUAL_DEVICES=8 timeout -k 10 300 $R --gpus 8 > gpurun_out/${T}_regime8.json 2> gpurun_out/${T}_regime8.err &&
NANOPOW_WATCHER=0 NANOPOW_VIRTUAL_DEVICES=8 timeout -k 10 300 $R --gpus 8 > gpurun_out/${T}_regime8_nowatch.json 2> gpurun_out/${T}_regime8_nowatch.err &&
NANOPOW_VIRTUAL_DEVICES=4 timeout -k 10 300 $R --gpus 4 > gpurun_out/${T}_regime4.json 2> gpurun_out/${T}_regime4.err &&
timeout -k 10 300 $R > gpurun_out/${T}_regime1.json 2> gpurun_out/${T}_regime1.err &&
NANOPOW_WATCHER=0 timeout -k 10 300 $R > gpurun_out/${T}_regime1_nowatch.json 2> gpurun_out/${T}_regime1_nowatch.err &&
timeout -k 10 900 $PYT tests -m gpu > gpurun_out/${T}_pytest_gpu.log 2>&1 &&
timeout -k 10 600 python3 tools/experiments/lib_arms_ab.py 3 watch=tree nowatch=tree@NANOPOW_WATCHER=0 > gpurun_out/${T}_ab_watcher.jsonl 2> gpurun_out/${T}_ab.err
rc=$?
tail -n 3 gpurun_out/${T}_pytest_gpu.log
exit $rc
