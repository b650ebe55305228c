#!/bin/bash
# Round-2 closing measurements on one GPU box (every GPU step under its own time limit, the chain
# stops at the first failure): GPU suite, smoke, the driver's bench command, the rocprofv3 kernel
# trace of the timed region, PMC traffic of the search kernel; with a second argument "workloads",
# every bench workload too (tools/workloads_refresh.sh; run it as its own call: gpurun's limit).
set -o pipefail
TAG=${1:-r02f}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_$TAG.log; exit 1; }
timeout -k 10 180 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || exit 1
timeout -k 10 400 python3 bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit 1
P="python3 bench.py --steps 100 --warmup 5 --no-cpu-baseline --latency-searches 0 --http-requests 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- $P > gpurun_out/bench_prof_$TAG.json 2> gpurun_out/prof_$TAG.err || exit 1
python3 tools/rocprof_timed_region.py gpurun_out/prof_$TAG/run_kernel_trace.csv gpurun_out/bench_prof_$TAG.json npow_pool_kernel_ls2_arg "rocprofv3 --kernel-trace --stats -- $P" > gpurun_out/timed_region_$TAG.txt || exit 1
bash tools/pmc_bench.sh $TAG npow_pool_kernel_ls2 gpurun_out/pmc_pool_$TAG.json -- --steps 100 --warmup 5 --latency-searches 0 || exit 1
[ "$2" = "workloads" ] && { bash tools/workloads_refresh.sh $TAG || exit 1; }
tail -2 gpurun_out/pytest_gpu_$TAG.log; cat gpurun_out/smoke_$TAG.log gpurun_out/timed_region_$TAG.txt
