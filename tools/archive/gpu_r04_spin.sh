#!/bin/bash
# Round 4: spinning-worker step gap A/B (tools/experiments/spin_ab.py); one step, its own time limit.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python3 tools/experiments/spin_ab.py run 2 tree gap2 gap5 gap10 > gpurun_out/r04_ab_spin.jsonl 2> gpurun_out/r04_ab_spin.err
rc=$?
cat gpurun_out/r04_ab_spin.jsonl; tail -3 gpurun_out/r04_ab_spin.err
exit $rc
