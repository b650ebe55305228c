#!/bin/bash
# Round-6 A/B under CPU contention (a shared host blocker behind the stop span's tail): the overshoot
# worker over 4 CU partitions, 600 receive-difficulty searches, pinned with 3 busy processes to 4 CPUs, with the
# final library (notifications sent after the pool lock is released) against a variant that sends them under it
# (build/v6, PoolLock without the deferral), interleaved, 3 runs each.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r06l}
O="python3 tests/overshoot_worker.py 600 receive"
pids=""
for i in 1 2 3; do taskset -c 0-3 timeout 300 python3 -c "while True: pass" & pids="$pids $!"; done
rc=0
for i in 1 2 3; do
  NANOPOW_VIRTUAL_DEVICES=4 timeout -k 10 100 taskset -c 0-3 $O > gpurun_out/${T}_defer_$i.json 2> gpurun_out/${T}_defer_$i.err || { rc=1; break; }
  NANOPOW_LIB=build/v6/nano-dpow_amd/nanopow/libnanopow.so NANOPOW_VIRTUAL_DEVICES=4 timeout -k 10 100 taskset -c 0-3 $O > gpurun_out/${T}_nodefer_$i.json 2> gpurun_out/${T}_nodefer_$i.err || { rc=1; break; }
done
kill $pids 2>/dev/null; wait 2>/dev/null
for f in gpurun_out/${T}_*.json; do python3 -c "
import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f'.split('/')[-1], d['stop_after_decide_us'], d['result_ms_p50'], d['finish_ms_p50'])"; done
exit $rc
