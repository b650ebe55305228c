#!/bin/bash
# Round 3: what the search loop's per-iteration s_barrier costs.  (1) the shipped stream in the
# two-group harness with a __syncthreads after every hash, none, or every 4th (stream_lockstep.py,
# LOCKSTEP_SYNC); (2) the search kernel with its loop barrier every 1 / 2 / 4 / 16 iterations
# (NPOW_LS2_EPOCH builds, setprio_ab.py), interleaved.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2 3; do for y in "" y0 y4; do timeout -k 5 60 ./build/stream_lockstep_g2$y || exit 1; done; done > gpurun_out/r03_sync_harness.jsonl &&
timeout -k 10 600 python3 tools/experiments/setprio_ab.py run 4 150 tree ep2 ep4 ep16 > gpurun_out/r03_ab_epoch.jsonl 2> gpurun_out/r03_ab_epoch.err
rc=$?
cat gpurun_out/r03_sync_harness.jsonl gpurun_out/r03_ab_epoch.jsonl; tail -3 gpurun_out/r03_ab_epoch.err
exit $rc
