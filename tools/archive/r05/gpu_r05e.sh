#!/bin/bash
# Round 5, session e: GPU-side timelines of first-found cancellation on CU partitions (NANOPOW_TRACE_LATENCY: each
# device's launch start / end on the GPU's realtime clock, from the deciding win) -- 8, 4 and 8 with 4 searching.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r05e}
O="timeout -k 10 200 python3 tests/overshoot_worker.py 100 receive"
NANOPOW_TRACE_LATENCY=1 NANOPOW_VIRTUAL_DEVICES=8 $O > gpurun_out/${T}_over_g8.json 2> gpurun_out/${T}_over_g8.err &&
NANOPOW_TRACE_LATENCY=1 NANOPOW_VIRTUAL_DEVICES=4 $O > gpurun_out/${T}_over_g4.json 2> gpurun_out/${T}_over_g4.err &&
NANOPOW_TRACE_LATENCY=1 NANOPOW_VIRTUAL_DEVICES=8 $O 0x55 > gpurun_out/${T}_over_g8_m55.json 2> gpurun_out/${T}_over_g8_m55.err
