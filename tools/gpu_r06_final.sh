#!/bin/bash
# Round-6 final GPU session on the final tree: the driver's commands (smoke, the whole GPU suite as the driver runs it,
# the bench with no flags and with --steps 20 --warmup 5), then the profiling recipe (tools/prof_r06.sh: the timed
# region with the regime child kept in, PMC passes of the search and sweep kernels, dual issue) whose files bench.py
# names in roofline.profile / roofline.traffic.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r06q}
bash tools/gpu_r06f.sh $T > gpurun_out/${T}_driver.log 2>&1 &&
bash tools/prof_r06.sh $T > gpurun_out/${T}_prof.log 2>&1
rc=$?
tail -6 gpurun_out/${T}_driver.log | cut -c1-400
grep -E "frac_executed|in_kernel_mhz|cycles_per_hash|agreement" gpurun_out/${T}_rocprofv3_timed_region.txt
exit $rc
