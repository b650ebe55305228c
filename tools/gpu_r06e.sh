#!/bin/bash
# Round-6 fifth GPU session: the exit tests (processes ending with launches in flight, plain and under rocprofv3),
# the round-4/5 profile recipe with the regime child left in (it crashed at exit under rocprofv3),
# then 6 more first-found-cancellation runs over 8 CU partitions with the stale-count classification.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r06e}
O="python3 tests/overshoot_worker.py 600 receive"
B="python3 bench.py --no-cpu-baseline --steps 100 --warmup 5 --latency-searches 0 --http-requests 0 --regime-searches 200"
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_exit.py -x -v --timeout 200 --timeout-method thread > gpurun_out/${T}_pytest_exit.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$T -o run -- $B > gpurun_out/${T}_prof_bench.json 2> gpurun_out/${T}_prof_bench.err &&
for i in 1 2 3 4 5 6; do NANOPOW_VIRTUAL_DEVICES=8 timeout -k 10 100 $O > gpurun_out/${T}_over8_$i.json 2> gpurun_out/${T}_over8_$i.err || exit 1; done
rc=$?
tail -12 gpurun_out/${T}_pytest_exit.log
echo "prof rc chain: $rc"; head -c 400 gpurun_out/${T}_prof_bench.json; echo
for f in gpurun_out/${T}_over8_*.json; do echo "$f"; python3 -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); print({k: d.get(k) for k in ('stop_after_decide_us','stale_drains','stale_late','stale_missing','stale_gpu_delay_us','linger_relays')})"; done
exit $rc
