#!/bin/bash
# Round 3: VGPR allocation order of the stream (gen_hash_asm.py --alloc low|high|rr): the same
# instructions and schedule on different registers -- does the power-limited clock move?
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 tools/experiments/setprio_ab.py run 4 150 tree al_high al_rr al_rr48 > gpurun_out/r03_ab_alloc.jsonl 2> gpurun_out/r03_ab_alloc.err
rc=$?
cat gpurun_out/r03_ab_alloc.jsonl; tail -3 gpurun_out/r03_ab_alloc.err
exit $rc
