#!/bin/bash
# Round 5, session t: the regime workload's host timeline with and without lingering, one device.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r05t}
L="python3 tools/experiments/regime_lat.py 1 600"
timeout -k 10 200 $L > gpurun_out/${T}_rlat.jsonl 2> gpurun_out/${T}_rlat.err &&
timeout -k 10 200 $L NANOPOW_LINGER=0 >> gpurun_out/${T}_rlat.jsonl 2>> gpurun_out/${T}_rlat.err &&
timeout -k 10 200 $L >> gpurun_out/${T}_rlat.jsonl 2>> gpurun_out/${T}_rlat.err &&
timeout -k 10 200 $L NANOPOW_LINGER=0 >> gpurun_out/${T}_rlat.jsonl 2>> gpurun_out/${T}_rlat.err
rc=$?
cat gpurun_out/${T}_rlat.jsonl
exit $rc
