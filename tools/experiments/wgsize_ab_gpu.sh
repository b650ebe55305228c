#!/bin/bash
# Round 3: the search kernel with 8 waves per SIMD in 1,024-lane workgroups (shipped), 512-lane (4 per
# CU) or 256-lane ones (8 per CU): NPOW_LS_WAVES builds (setprio_ab.py), interleaved.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 tools/experiments/setprio_ab.py run 4 150 tree w8 w4 > gpurun_out/r03_ab_wgsize.jsonl 2> gpurun_out/r03_ab_wgsize.err
rc=$?
cat gpurun_out/r03_ab_wgsize.jsonl; tail -3 gpurun_out/r03_ab_wgsize.err
exit $rc
