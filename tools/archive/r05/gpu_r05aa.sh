#!/bin/bash
# Round 5, session aa: polls read dynamic entries past the caches (no acquire in polls) -- linger tests, overshoot over
# 8 / 4 partitions, the join spread (diagnostic library), the regime A/B over 1 / 8 devices and the bench A/B.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r05aa}
PYT="python3 -u -m pytest -x -v --timeout 120 --timeout-method thread"
timeout -k 10 300 $PYT tests/test_gpu_linger.py > gpurun_out/${T}_linger.log 2>&1 &&
NANOPOW_TEST_HOOKS=1 NANOPOW_VIRTUAL_DEVICES=8 timeout -k 10 200 python3 tests/overshoot_worker.py 200 receive > gpurun_out/${T}_over_g8.json 2> gpurun_out/${T}_over_g8.err &&
NANOPOW_TEST_HOOKS=1 NANOPOW_VIRTUAL_DEVICES=4 timeout -k 10 200 python3 tests/overshoot_worker.py 200 receive > gpurun_out/${T}_over_g4.json 2> gpurun_out/${T}_over_g4.err &&
NANOPOW_LIB=$PWD/build/diag/libnanopow.so LAT_STDERR=gpurun_out/${T}_serial.err timeout -k 10 120 python3 tools/experiments/lat_fields.py 150 ffffffc000000000 > gpurun_out/${T}_serial.json 2>&1 &&
timeout -k 10 700 python3 tools/experiments/regime_ab.py 2 1000 l1=1 n1=1@NANOPOW_LINGER=0 l8=8 n8=8@NANOPOW_LINGER=0 > gpurun_out/${T}_regime_ab.jsonl 2> gpurun_out/${T}_regime_ab.err &&
timeout -k 10 600 python3 tools/experiments/lib_arms_ab.py 2 tree=tree nl=tree@NANOPOW_LINGER=0 > gpurun_out/${T}_ab.jsonl 2> gpurun_out/${T}_ab.err
rc=$?
tail -n 2 gpurun_out/${T}_linger.log
grep -o '"stop_after_decide_us": {[^}]*}' gpurun_out/${T}_over_g*.json
exit $rc
