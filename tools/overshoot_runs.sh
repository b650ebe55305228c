#!/bin/bash
# The first-found cancellation worker (tests/overshoot_worker.py, 200 receive-difficulty searches) N times over 8 and
# over 4 CU partitions: the distribution of the losers' stop span behind the bounds in tests/test_gpu_multidevice.py.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-ovr}; N=${2:-5}
for r in $(seq 1 $N); do
  for g in 8 4; do
    NANOPOW_TEST_HOOKS=1 NANOPOW_VIRTUAL_DEVICES=$g timeout -k 10 120 python3 tests/overshoot_worker.py 200 receive > gpurun_out/${T}_g${g}_$r.json 2> gpurun_out/${T}_g${g}_$r.err || exit 1
    echo "g$g $r $(grep -o '"stop_after_decide_us": {[^}]*}' gpurun_out/${T}_g${g}_$r.json)"
  done
done
