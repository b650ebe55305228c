#!/bin/bash
# Round-5 re-close after the lingering default moved to CU partitions of <= 32 CUs: the GPU suite, the closing bench
# session (tools/final_r05.sh) and the profiles of this build (tools/prof_r04.sh).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r05g}
timeout -k 10 420 python3 -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1 &&
bash tools/final_r05.sh $T &&
bash tools/prof_r04.sh $T > gpurun_out/${T}_prof.log 2>&1
