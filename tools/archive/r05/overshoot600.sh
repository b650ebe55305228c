#!/bin/bash
# Round 5: the first-found stop span over 600 searches per run (p99 = the 6th largest), 6 runs over 8 and 4 CU
# partitions with the default lingering policy -- the distribution behind tests/test_gpu_multidevice.py's bounds.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-o600}
for r in 1 2 3 4 5 6; do
  for g in 8 4; do
    NANOPOW_TEST_HOOKS=1 NANOPOW_VIRTUAL_DEVICES=$g timeout -k 10 120 python3 tests/overshoot_worker.py 600 receive > gpurun_out/${T}_g${g}_$r.json 2> gpurun_out/${T}_g${g}_$r.err || exit 1
    echo "g$g $r $(grep -o '"stop_after_decide_us": {[^}]*}' gpurun_out/${T}_g${g}_$r.json)"
  done
done
