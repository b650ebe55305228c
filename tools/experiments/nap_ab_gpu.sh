#!/bin/bash
# Round 3: the pool worker's nap between polls (NANOPOW_POLL_US, default 50 us; 0 = spin) on serial
# send-difficulty searches -- the GPU idles between one search's win and the next one's launch.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 tools/experiments/setprio_ab.py run 4 150 tree NANOPOW_POLL_US=20 NANOPOW_POLL_US=0 > gpurun_out/r03_ab_nap.jsonl 2> gpurun_out/r03_ab_nap.err
rc=$?
cat gpurun_out/r03_ab_nap.jsonl; tail -3 gpurun_out/r03_ab_nap.err
exit $rc
