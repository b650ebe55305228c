#!/bin/bash
# One GPU-box session: GPU tests, smoke, bench, rocprofv3 kernel stats.  Every GPU step has its own
# time limit and the chain stops at the first failure.
set -o pipefail
TAG=${1:-r01}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1 &&
timeout -k 10 180 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 &&
timeout -k 10 400 python3 bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python3 bench.py --no-cpu-baseline --steps 200 > gpurun_out/bench_prof_$TAG.json 2> gpurun_out/prof_$TAG.err
rc=$?
tail -3 gpurun_out/pytest_gpu_$TAG.log; cat gpurun_out/smoke_$TAG.log gpurun_out/bench_$TAG.json 2>/dev/null
exit $rc
