#!/bin/bash
# Round-6 first GPU session: smoke, the whole GPU suite in its new order (parity and the JSON drop-in first, latency
# last), then an interleaved A/B of the default bench line against the round-5 library (build/base_r05) -- the
# kernel's lingering path and the host's watcher / waiter spin windows changed.  Every GPU step has its own time
# limit; the chain stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r06b}
B="python3 bench.py --no-cpu-baseline --steps 100 --warmup 5 --latency-searches 300 --http-requests 0 --regime-searches 0"
timeout -k 10 180 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 &&
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_exit.py -x -v --timeout 200 --timeout-method thread > gpurun_out/${T}_pytest_exit.log 2>&1 &&
timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread --ignore=tests/test_gpu_exit.py > gpurun_out/${T}_pytest_gpu.log 2>&1 &&
timeout -k 10 120 $B > gpurun_out/${T}_bench_new1.json 2> gpurun_out/${T}_bench_new1.err &&
NANOPOW_LIB=build/base_r05/libnanopow.so timeout -k 10 120 $B > gpurun_out/${T}_bench_base1.json 2> gpurun_out/${T}_bench_base1.err &&
timeout -k 10 120 $B > gpurun_out/${T}_bench_new2.json 2> gpurun_out/${T}_bench_new2.err &&
NANOPOW_LIB=build/base_r05/libnanopow.so timeout -k 10 120 $B > gpurun_out/${T}_bench_base2.json 2> gpurun_out/${T}_bench_base2.err
rc=$?
tail -5 gpurun_out/${T}_pytest_exit.log gpurun_out/${T}_pytest_gpu.log
for f in gpurun_out/${T}_bench_*.json; do echo "$f"; head -c 400 "$f"; echo; done
exit $rc
