#!/bin/bash
# Round 3: 512-lane workgroups (NPOW_LS_WAVES=8 build) against the shipped 1,024-lane ones beyond the
# search rate: 2^34 sweeps (exact) and per-search latency, interleaved.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
W8=NANOPOW_LIB=$PWD/build/abprio/w8/libnanopow.so
timeout -k 10 300 python3 tools/experiments/sweep_groups_ab.py 3 NANOPOW_POLL=1024 $W8 > gpurun_out/r03_ab_wgsize_sweep.jsonl 2> gpurun_out/r03_ab_wgsize_sweep.err &&
timeout -k 10 400 python3 tools/experiments/latency_ab.py 4 200 tree w8 > gpurun_out/r03_ab_wgsize_latency.jsonl 2> gpurun_out/r03_ab_wgsize_latency.err
rc=$?
cat gpurun_out/r03_ab_wgsize_sweep.jsonl gpurun_out/r03_ab_wgsize_latency.jsonl; tail -3 gpurun_out/r03_ab_wgsize_*.err
exit $rc
