#!/bin/bash
# Round 5, sessions j-k: lingering launches (a search launch waits in the GPU for the next dynamic entry) -- their tests,
# the GPU suite, the bench / receive A/B against NANOPOW_LINGER=0, the regime A/B over 1 and 8 devices, the overshoot
# worker over 8 and 4 CU partitions.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r05j}
PYT="python3 -u -m pytest -x -v --timeout 120 --timeout-method thread"
timeout -k 10 300 $PYT tests/test_gpu_linger.py > gpurun_out/${T}_linger.log 2>&1 &&
timeout -k 10 400 $PYT tests/test_gpu_multidevice.py > gpurun_out/${T}_multidevice.log 2>&1 &&
timeout -k 10 900 $PYT tests -m gpu > gpurun_out/${T}_pytest_gpu.log 2>&1 &&
timeout -k 10 600 python3 tools/experiments/lib_arms_ab.py 3 tree=tree nl=tree@NANOPOW_LINGER=0 > gpurun_out/${T}_ab.jsonl 2> gpurun_out/${T}_ab.err &&
timeout -k 10 600 python3 tools/experiments/regime_ab.py 2 1000 l1=1 n1=1@NANOPOW_LINGER=0 l8=8 n8=8@NANOPOW_LINGER=0 > gpurun_out/${T}_regime_ab.jsonl 2> gpurun_out/${T}_regime_ab.err &&
NANOPOW_TEST_HOOKS=1 NANOPOW_VIRTUAL_DEVICES=8 timeout -k 10 200 python3 tests/overshoot_worker.py 200 receive > gpurun_out/${T}_over_g8.json 2> gpurun_out/${T}_over_g8.err &&
NANOPOW_TEST_HOOKS=1 NANOPOW_VIRTUAL_DEVICES=4 timeout -k 10 200 python3 tests/overshoot_worker.py 200 receive > gpurun_out/${T}_over_g4.json 2> gpurun_out/${T}_over_g4.err
rc=$?
tail -n 5 gpurun_out/${T}_linger.log; tail -n 3 gpurun_out/${T}_pytest_gpu.log
exit $rc
