#!/bin/bash
# Round 5, session h: slots finished from their final count freed without a read-back -- the GPU suite, then the
# regime interleaved with NANOPOW_READBACK=always over 1 / 4 / 8 devices, the overshoot worker on 8 and 4.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r05h}
PYT="python3 -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 900 $PYT tests -m gpu > gpurun_out/${T}_pytest_gpu.log 2>&1 &&
timeout -k 10 600 python3 tools/experiments/regime_ab.py 2 1000 n1=1 rb1=1@NANOPOW_READBACK=always n4=4 rb4=4@NANOPOW_READBACK=always n8=8 rb8=8@NANOPOW_READBACK=always > gpurun_out/${T}_regime_ab.jsonl 2> gpurun_out/${T}_regime_ab.err &&
NANOPOW_TEST_HOOKS=1 NANOPOW_VIRTUAL_DEVICES=8 timeout -k 10 200 python3 tests/overshoot_worker.py 200 receive > gpurun_out/${T}_over_g8.json 2> gpurun_out/${T}_over_g8.err &&
NANOPOW_TEST_HOOKS=1 NANOPOW_VIRTUAL_DEVICES=4 timeout -k 10 200 python3 tests/overshoot_worker.py 200 receive > gpurun_out/${T}_over_g4.json 2> gpurun_out/${T}_over_g4.err
rc=$?
tail -n 3 gpurun_out/${T}_pytest_gpu.log
exit $rc
