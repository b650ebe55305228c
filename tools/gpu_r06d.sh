#!/bin/bash
# Round-6 fourth GPU session: first-found cancellation over CU partitions with the stale-count classification
# (3 runs over 8 partitions, lingering by default; 2 over 4 with lingering forced on), the A/B of the default bench
# line against the round-5 library, the GPU suite without the exit tests, then the exit diagnosis under rocprofv3
# (last: a crash or hang there ends the call).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r06d}
B="python3 bench.py --no-cpu-baseline --steps 100 --warmup 5 --latency-searches 300 --http-requests 0 --regime-searches 0"
P="rocprofv3 --kernel-trace --stats --output-format csv"
O="python3 tests/overshoot_worker.py 600 receive"
timeout -k 10 180 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 &&
NANOPOW_VIRTUAL_DEVICES=8 timeout -k 10 100 $O > gpurun_out/${T}_over8_1.json 2> gpurun_out/${T}_over8_1.err &&
NANOPOW_VIRTUAL_DEVICES=8 timeout -k 10 100 $O > gpurun_out/${T}_over8_2.json 2> gpurun_out/${T}_over8_2.err &&
NANOPOW_VIRTUAL_DEVICES=8 timeout -k 10 100 $O > gpurun_out/${T}_over8_3.json 2> gpurun_out/${T}_over8_3.err &&
NANOPOW_LINGER=1 NANOPOW_VIRTUAL_DEVICES=4 timeout -k 10 100 $O > gpurun_out/${T}_over4L_1.json 2> gpurun_out/${T}_over4L_1.err &&
NANOPOW_LINGER=1 NANOPOW_VIRTUAL_DEVICES=4 timeout -k 10 100 $O > gpurun_out/${T}_over4L_2.json 2> gpurun_out/${T}_over4L_2.err &&
timeout -k 10 120 $B > gpurun_out/${T}_bench_new1.json 2> gpurun_out/${T}_bench_new1.err &&
NANOPOW_LIB=build/base_r05/libnanopow.so timeout -k 10 120 $B > gpurun_out/${T}_bench_base1.json 2> gpurun_out/${T}_bench_base1.err &&
timeout -k 10 120 $B > gpurun_out/${T}_bench_new2.json 2> gpurun_out/${T}_bench_new2.err &&
NANOPOW_LIB=build/base_r05/libnanopow.so timeout -k 10 120 $B > gpurun_out/${T}_bench_base2.json 2> gpurun_out/${T}_bench_base2.err &&
timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread --ignore=tests/test_gpu_exit.py > gpurun_out/${T}_pytest_gpu.log 2>&1 &&
NANOPOW_VIRTUAL_DEVICES=8 timeout -s KILL 100 $P -d /tmp/${T}_o8 -o run -- python3 tests/overshoot_worker.py 100 receive > gpurun_out/${T}_exit_over8.json 2> gpurun_out/${T}_exit_over8.err &&
NANOPOW_VIRTUAL_DEVICES=8 timeout -s KILL 100 $P -d /tmp/${T}_rg -o run -- python3 bench.py --workload regime --gpus 8 --steps 200 --http-requests 20 > gpurun_out/${T}_exit_regime.json 2> gpurun_out/${T}_exit_regime.err
rc=$?
for f in gpurun_out/${T}_over*.json; do echo "$f"; python3 -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); print({k: d.get(k) for k in ('stop_after_decide_us','stale_drains','stale_late','stale_missing','stale_gpu_delay_us','linger_relays')})"; done
tail -3 gpurun_out/${T}_pytest_gpu.log
for f in gpurun_out/${T}_bench_*.json; do echo "$f"; head -c 300 "$f"; echo; done
tail -c 1500 gpurun_out/${T}_exit_over8.err; echo; tail -c 3000 gpurun_out/${T}_exit_regime.err
exit $rc
