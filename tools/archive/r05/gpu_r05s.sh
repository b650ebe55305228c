#!/bin/bash
# Round 5, session s: the host timeline of serial searches with and without lingering (one device, 2^26-nonce
# searches; 8 CU partitions).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r05s}
L="python3 tools/experiments/lat_fields.py 400 ffffffc000000000"
timeout -k 10 200 $L > gpurun_out/${T}_lat.jsonl 2> gpurun_out/${T}_lat.err &&
timeout -k 10 200 $L NANOPOW_LINGER=0 >> gpurun_out/${T}_lat.jsonl 2>> gpurun_out/${T}_lat.err &&
timeout -k 10 200 $L NANOPOW_VIRTUAL_DEVICES=8 >> gpurun_out/${T}_lat.jsonl 2>> gpurun_out/${T}_lat.err &&
timeout -k 10 200 $L NANOPOW_VIRTUAL_DEVICES=8 NANOPOW_LINGER=0 >> gpurun_out/${T}_lat.jsonl 2>> gpurun_out/${T}_lat.err
rc=$?
cat gpurun_out/${T}_lat.jsonl
exit $rc
