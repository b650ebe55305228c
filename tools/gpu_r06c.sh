#!/bin/bash
# Round-6 third GPU session: the GPU suite without the exit tests, the A/B of the default bench line against the
# round-5 library, then the exit diagnosis (last: a crash or hang there ends the call) -- the overshoot worker over 8
# CU partitions under rocprofv3 (8 streams over the box's 4 hardware queues), then the bench's regime child, with its
# whole stderr kept.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r06c}
B="python3 bench.py --no-cpu-baseline --steps 100 --warmup 5 --latency-searches 300 --http-requests 0 --regime-searches 0"
P="rocprofv3 --kernel-trace --stats --output-format csv"
timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread --ignore=tests/test_gpu_exit.py > gpurun_out/${T}_pytest_gpu.log 2>&1 &&
timeout -k 10 120 $B > gpurun_out/${T}_bench_new1.json 2> gpurun_out/${T}_bench_new1.err &&
NANOPOW_LIB=build/base_r05/libnanopow.so timeout -k 10 120 $B > gpurun_out/${T}_bench_base1.json 2> gpurun_out/${T}_bench_base1.err &&
timeout -k 10 120 $B > gpurun_out/${T}_bench_new2.json 2> gpurun_out/${T}_bench_new2.err &&
NANOPOW_LIB=build/base_r05/libnanopow.so timeout -k 10 120 $B > gpurun_out/${T}_bench_base2.json 2> gpurun_out/${T}_bench_base2.err &&
NANOPOW_VIRTUAL_DEVICES=8 timeout -s KILL 100 $P -d /tmp/${T}_o8 -o run -- python3 tests/overshoot_worker.py 100 receive > gpurun_out/${T}_exit_over8.json 2> gpurun_out/${T}_exit_over8.err &&
NANOPOW_VIRTUAL_DEVICES=8 timeout -s KILL 100 $P -d /tmp/${T}_rg -o run -- python3 bench.py --workload regime --gpus 8 --steps 200 --http-requests 20 > gpurun_out/${T}_exit_regime.json 2> gpurun_out/${T}_exit_regime.err
rc=$?
tail -3 gpurun_out/${T}_pytest_gpu.log
for f in gpurun_out/${T}_bench_*.json; do echo "$f"; head -c 300 "$f"; echo; done
tail -c 1500 gpurun_out/${T}_exit_over8.err; echo; tail -c 3000 gpurun_out/${T}_exit_regime.err
exit $rc
