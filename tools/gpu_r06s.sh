#!/bin/bash
# Round-6 long runs on the final build: a 10-minute pool soak over 8 CU partitions (lingering launches by default
# there; every result checked), then 10 more runs of 600 first-found-cancellation searches over 8 partitions with the
# stale final-count classification.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r06s}
NANOPOW_VIRTUAL_DEVICES=8 timeout -k 10 700 python3 -u tools/pool_soak.py --seconds 600 > gpurun_out/${T}_soak8_600s.log 2>&1 &&
for i in 1 2 3 4 5 6 7 8 9 10; do NANOPOW_VIRTUAL_DEVICES=8 timeout -k 10 100 python3 tests/overshoot_worker.py 600 receive > gpurun_out/${T}_over8_$i.json 2> gpurun_out/${T}_over8_$i.err || exit 1; done
rc=$?
tail -1 gpurun_out/${T}_soak8_600s.log | cut -c1-400
for f in gpurun_out/${T}_over8_*.json; do python3 -c "import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f'.split('/')[-1], d['stop_after_decide_us'], {k: d.get(k) for k in ('stale_drains','stale_late','stale_missing','linger_relays')})"; done
exit $rc
