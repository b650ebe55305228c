#!/bin/bash
# Round-4 profiles of the default bench workload: rocprofv3 kernel trace + stats (timed-region average
# against the bench's HIP-event average, the roofline fraction recomputed from it, the build's build_sha16),
# then PMC passes for the search kernel and the sweep kernel, and the dual-issue pass.
# (--regime-searches 0: the 2^26 regime leg runs in a child process, which crashed with SIGSEGV in its exit
# handlers under rocprofv3 in round 5 -- after the timed region, but its error then stood in the profiled line)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r04}
B="python3 bench.py --no-cpu-baseline --steps 100 --warmup 5 --latency-searches 0 --http-requests 0 --regime-searches 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- $B > gpurun_out/prof_${TAG}_bench.json 2> gpurun_out/prof_${TAG}.err &&
python3 tools/rocprof_timed_region.py gpurun_out/prof_$TAG/run_kernel_trace.csv gpurun_out/prof_${TAG}_bench.json npow_pool_kernel_ls2_arg "$B" > gpurun_out/${TAG}_rocprofv3_timed_region.txt &&
bash tools/pmc_bench.sh ${TAG}pool npow_pool_kernel_ls2 gpurun_out/${TAG}_pmc_pool.json -- --steps 100 --warmup 5 --latency-searches 0 --regime-searches 0 &&
bash tools/pmc_bench.sh ${TAG}sweep npow_sweep_kernel_ls2 gpurun_out/${TAG}_pmc_sweep.json -- --workload sweep --sweep-bits 35 --regime-searches 0 &&
bash tools/pmc_dual_issue.sh $TAG
rc=$?
cat gpurun_out/${TAG}_rocprofv3_timed_region.txt; head -c 1500 gpurun_out/${TAG}_pmc_pool.json; head -c 800 gpurun_out/${TAG}_pmc_sweep.json
exit $rc
