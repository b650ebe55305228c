#!/bin/bash
# Round 5, session m: the host worker's step profile (NANOPOW_TRACE_STEPS) under the 4-partition overshoot run,
# lingering on and off.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r05m}
O="python3 tests/overshoot_worker.py 400 receive"
NANOPOW_TRACE_STEPS=1 NANOPOW_TEST_HOOKS=1 NANOPOW_VIRTUAL_DEVICES=${G:-4} timeout -k 10 200 $O > gpurun_out/${T}_over_g4.json 2> gpurun_out/${T}_over_g4.err &&
NANOPOW_LINGER=0 NANOPOW_TRACE_STEPS=1 NANOPOW_TEST_HOOKS=1 NANOPOW_VIRTUAL_DEVICES=${G:-4} timeout -k 10 200 $O > gpurun_out/${T}_over_g4_nl.json 2> gpurun_out/${T}_over_g4_nl.err
rc=$?
grep -o '"stop_after_decide_us": {[^}]*}' gpurun_out/${T}_over_g4*.json
grep "nanopow-steps\[0\]" gpurun_out/${T}_over_g4.err gpurun_out/${T}_over_g4_nl.err
exit $rc
