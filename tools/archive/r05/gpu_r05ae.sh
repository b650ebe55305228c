#!/bin/bash
# Round 5, session ae: per-workgroup acquires again (picks only), lingering by default with 2+ GPU devices -- the
# linger tests, overshoot over 8 / 4 partitions, the GPU suite, the regime A/B.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r05ae}
PYT="python3 -u -m pytest -x -v --timeout 120 --timeout-method thread"
O="python3 tests/overshoot_worker.py 200 receive"
timeout -k 10 300 $PYT tests/test_gpu_linger.py > gpurun_out/${T}_linger.log 2>&1 || exit 1
for r in 1 2; do
  NANOPOW_TEST_HOOKS=1 NANOPOW_VIRTUAL_DEVICES=8 timeout -k 10 120 $O > gpurun_out/${T}_g8_$r.json 2> gpurun_out/${T}_g8_$r.err || exit 1
  echo "g8 $r $(grep -o '"stop_after_decide_us": {[^}]*}' gpurun_out/${T}_g8_$r.json)"
  NANOPOW_TEST_HOOKS=1 NANOPOW_VIRTUAL_DEVICES=4 timeout -k 10 120 $O > gpurun_out/${T}_g4_$r.json 2> gpurun_out/${T}_g4_$r.err || exit 1
  echo "g4 $r $(grep -o '"stop_after_decide_us": {[^}]*}' gpurun_out/${T}_g4_$r.json)"
done
timeout -k 10 900 $PYT tests -m gpu > gpurun_out/${T}_pytest_gpu.log 2>&1 &&
timeout -k 10 700 python3 tools/experiments/regime_ab.py 2 1000 d1=1 l1=1@NANOPOW_LINGER=1 l8=8 n8=8@NANOPOW_LINGER=0 > gpurun_out/${T}_regime_ab.jsonl 2> gpurun_out/${T}_regime_ab.err
rc=$?
tail -n 1 gpurun_out/${T}_linger.log; tail -n 2 gpurun_out/${T}_pytest_gpu.log
exit $rc
