#!/bin/bash
# Round-3 GPU session: smoke, the changed GPU tests first, then the whole GPU suite and the default
# bench line.  Every GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
TAG=${1:-r03}
mkdir -p gpurun_out
export TMPDIR=/tmp
PYT="python3 -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 180 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 &&
timeout -k 10 600 $PYT -s tests/test_gpu_parity.py tests/test_gpu_kernels.py tests/test_gpu_multidevice.py > gpurun_out/pytest_new_$TAG.log 2>&1 &&
timeout -k 10 900 $PYT tests -m gpu --deselect tests/test_gpu_parity.py --deselect tests/test_gpu_kernels.py --deselect tests/test_gpu_multidevice.py > gpurun_out/pytest_rest_$TAG.log 2>&1 &&
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?
tail -3 gpurun_out/smoke_$TAG.log gpurun_out/pytest_new_$TAG.log gpurun_out/pytest_rest_$TAG.log 2>/dev/null; cat gpurun_out/bench_$TAG.json 2>/dev/null | head -c 3000
exit $rc
