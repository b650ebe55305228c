#!/bin/bash
# Round-6: the rocprofv3 timed-region profile of the final build again (tools/prof_r06.sh's first two steps only:
# part 2 ran on a box whose kernel clock was 2,000 MHz) -- the bench's roofline.profile cross-check.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r06p}
B="python3 bench.py --no-cpu-baseline --steps 100 --warmup 5 --latency-searches 0 --http-requests 0 --regime-searches 200"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- $B > gpurun_out/prof_${TAG}_bench.json 2> gpurun_out/prof_${TAG}.err &&
python3 tools/rocprof_timed_region.py gpurun_out/prof_$TAG/run_kernel_trace.csv gpurun_out/prof_${TAG}_bench.json npow_pool_kernel_ls2_arg "$B" > gpurun_out/${TAG}_rocprofv3_timed_region.txt
rc=$?
cat gpurun_out/${TAG}_rocprofv3_timed_region.txt
exit $rc
