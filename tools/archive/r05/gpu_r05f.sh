#!/bin/bash
# Round 5, session f: where the 8-partition stop goes on the GPU (a diagnostic build that also stamps the kill's
# relay): relay / final count / host view from the deciding win, 8 and 4 partitions.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r05f}
O="timeout -k 10 200 python3 tests/overshoot_worker.py 100 receive"
NANOPOW_LIB=build/diag/libnanopow.so NANOPOW_TRACE_LATENCY=1 NANOPOW_VIRTUAL_DEVICES=8 $O > gpurun_out/${T}_over_g8.json 2> gpurun_out/${T}_over_g8.err &&
NANOPOW_LIB=build/diag/libnanopow.so NANOPOW_TRACE_LATENCY=1 NANOPOW_VIRTUAL_DEVICES=4 $O > gpurun_out/${T}_over_g4.json 2> gpurun_out/${T}_over_g4.err
