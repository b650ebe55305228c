#!/bin/bash
# Round 5, session af: one elected L2 invalidation per XCD, picks reading headers past the caches -- overshoot over 8
# (3 runs) and 4 partitions, the join spread on one device (diagnostic library, lingering forced on), the linger tests,
# the regime A/B (one device with lingering forced on, 8 partitions) and the bench / receive A/B.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r05af}
O="python3 tests/overshoot_worker.py 200 receive"
for r in 1 2 3; do
  NANOPOW_TEST_HOOKS=1 NANOPOW_VIRTUAL_DEVICES=8 timeout -k 10 120 $O > gpurun_out/${T}_g8_$r.json 2> gpurun_out/${T}_g8_$r.err || exit 1
  echo "g8 $r $(grep -o '"stop_after_decide_us": {[^}]*}' gpurun_out/${T}_g8_$r.json)"
done
NANOPOW_TEST_HOOKS=1 NANOPOW_VIRTUAL_DEVICES=4 timeout -k 10 120 $O > gpurun_out/${T}_g4.json 2> gpurun_out/${T}_g4.err || exit 1
echo "g4 $(grep -o '"stop_after_decide_us": {[^}]*}' gpurun_out/${T}_g4.json)"
NANOPOW_LINGER=1 NANOPOW_LIB=$PWD/build/diag/libnanopow.so LAT_STDERR=gpurun_out/${T}_serial.err timeout -k 10 120 python3 tools/experiments/lat_fields.py 150 ffffffc000000000 > gpurun_out/${T}_serial.json 2>&1 &&
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_linger.py > gpurun_out/${T}_linger.log 2>&1 &&
timeout -k 10 700 python3 tools/experiments/regime_ab.py 2 1000 d1=1 l1=1@NANOPOW_LINGER=1 l8=8 > gpurun_out/${T}_regime_ab.jsonl 2> gpurun_out/${T}_regime_ab.err &&
timeout -k 10 600 python3 tools/experiments/lib_arms_ab.py 2 d1=tree l1=tree@NANOPOW_LINGER=1 > gpurun_out/${T}_ab.jsonl 2> gpurun_out/${T}_ab.err
rc=$?
tail -n 1 gpurun_out/${T}_linger.log
exit $rc
