#!/bin/bash
# Round 5, session q: the replacement lingering launch queued at once -- the yielded-launch probe over 8 partitions,
# the overshoot worker over 8 and 4 partitions (timestamped debug log on 8), then the linger tests and the GPU suite.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r05q}
PYT="python3 -u -m pytest -x -v --timeout 120 --timeout-method thread"
NANOPOW_DEBUG=1 NANOPOW_VIRTUAL_DEVICES=8 timeout -k 10 120 python3 tools/experiments/linger_probe.py 3 70 > gpurun_out/${T}_probe8.txt 2> gpurun_out/${T}_probe8.err &&
NANOPOW_DEBUG=1 NANOPOW_TRACE_LATENCY=1 NANOPOW_TEST_HOOKS=1 NANOPOW_VIRTUAL_DEVICES=8 timeout -k 10 200 python3 tests/overshoot_worker.py 200 receive > gpurun_out/${T}_over_g8_dbg.json 2> gpurun_out/${T}_over_g8_dbg.err &&
NANOPOW_TEST_HOOKS=1 NANOPOW_VIRTUAL_DEVICES=8 timeout -k 10 200 python3 tests/overshoot_worker.py 200 receive > gpurun_out/${T}_over_g8.json 2> gpurun_out/${T}_over_g8.err &&
NANOPOW_TEST_HOOKS=1 NANOPOW_VIRTUAL_DEVICES=4 timeout -k 10 200 python3 tests/overshoot_worker.py 200 receive > gpurun_out/${T}_over_g4.json 2> gpurun_out/${T}_over_g4.err &&
timeout -k 10 300 $PYT tests/test_gpu_linger.py > gpurun_out/${T}_linger.log 2>&1 &&
timeout -k 10 900 $PYT tests -m gpu > gpurun_out/${T}_pytest_gpu.log 2>&1
rc=$?
cat gpurun_out/${T}_probe8.txt
grep -o '"stop_after_decide_us": {[^}]*}' gpurun_out/${T}_over_g*.json
tail -n 2 gpurun_out/${T}_linger.log; tail -n 2 gpurun_out/${T}_pytest_gpu.log
exit $rc
