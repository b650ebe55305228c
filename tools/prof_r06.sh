#!/bin/bash
# Round-6 profiles of the default bench workload (tools/prof_r04.sh with the regime child kept in the profiled
# bench: the exit-time SIGSEGV it had under rocprofv3 is fixed): rocprofv3 kernel trace + stats (timed-region average
# against the bench's HIP-event average, the roofline fraction recomputed from it, the build's build_sha16),
# then PMC passes for the search kernel and the sweep kernel, and the dual-issue pass.
# (The PMC passes still skip the regime leg: it is not what they measure.)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r06}
B="python3 bench.py --no-cpu-baseline --steps 100 --warmup 5 --latency-searches 0 --http-requests 0 --regime-searches 200"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- $B > gpurun_out/prof_${TAG}_bench.json 2> gpurun_out/prof_${TAG}.err &&
python3 tools/rocprof_timed_region.py gpurun_out/prof_$TAG/run_kernel_trace.csv gpurun_out/prof_${TAG}_bench.json npow_pool_kernel_ls2_arg "$B" > gpurun_out/${TAG}_rocprofv3_timed_region.txt &&
bash tools/pmc_bench.sh ${TAG}pool npow_pool_kernel_ls2 gpurun_out/${TAG}_pmc_pool.json -- --steps 100 --warmup 5 --latency-searches 0 --regime-searches 0 &&
bash tools/pmc_bench.sh ${TAG}sweep npow_sweep_kernel_ls2 gpurun_out/${TAG}_pmc_sweep.json -- --workload sweep --sweep-bits 35 --regime-searches 0 &&
bash tools/pmc_dual_issue.sh $TAG
rc=$?
cat gpurun_out/${TAG}_rocprofv3_timed_region.txt; head -c 1500 gpurun_out/${TAG}_pmc_pool.json; head -c 800 gpurun_out/${TAG}_pmc_sweep.json
exit $rc
