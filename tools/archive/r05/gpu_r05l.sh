#!/bin/bash
# Round 5, session l: the overshoot worker over 4 CU partitions with NANOPOW_TRACE_LATENCY (per-search fin / relay
# timelines, slots stopped without a final count), lingering on and off.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r05l}
O="python3 tests/overshoot_worker.py 400 receive"
NANOPOW_TRACE_LATENCY=1 NANOPOW_TEST_HOOKS=1 NANOPOW_VIRTUAL_DEVICES=4 timeout -k 10 200 $O > gpurun_out/${T}_over_g4.json 2> gpurun_out/${T}_over_g4.err &&
NANOPOW_LINGER=0 NANOPOW_TRACE_LATENCY=1 NANOPOW_TEST_HOOKS=1 NANOPOW_VIRTUAL_DEVICES=4 timeout -k 10 200 $O > gpurun_out/${T}_over_g4_nl.json 2> gpurun_out/${T}_over_g4_nl.err
rc=$?
grep -o '"stop_after_decide_us": {[^}]*}' gpurun_out/${T}_over_g4*.json
grep -c nofin gpurun_out/${T}_over_g4.err gpurun_out/${T}_over_g4_nl.err
exit $rc
