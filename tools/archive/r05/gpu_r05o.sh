#!/bin/bash
# Round 5, session o: the 8-partition overshoot run with the pool's timestamped debug log and the fin timelines.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r05o}
NANOPOW_DEBUG=1 NANOPOW_TRACE_LATENCY=1 NANOPOW_TEST_HOOKS=1 NANOPOW_VIRTUAL_DEVICES=8 timeout -k 10 200 python3 tests/overshoot_worker.py 200 receive > gpurun_out/${T}_over_g8.json 2> gpurun_out/${T}_over_g8.err
rc=$?
grep -o '"stop_after_decide_us": {[^}]*}' gpurun_out/${T}_over_g8.json
exit $rc
