#!/bin/bash
# Round 4: does the host-observed stop span over 8 CU partitions depend on how many hardware queues HIP
# opens (GPU_MAX_HW_QUEUES, 4 on the box)?  The overshoot worker (100 receive-difficulty searches split over
# 8 partitions) under 2, 4 and 8 queues, twice, each its own process and time limit.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=gpurun_out/r04_hwq_overshoot.jsonl
: > $OUT
for r in 0 1; do
  for q in 2 4 8; do
    GPU_MAX_HW_QUEUES=$q NANOPOW_VIRTUAL_DEVICES=8 timeout -k 10 120 python3 tests/overshoot_worker.py 100 receive > gpurun_out/hwq_$q.json 2> gpurun_out/hwq_$q.err || exit $?
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/hwq_$q.json').read().strip().splitlines()[-1]); print(json.dumps({'hw_queues': $q, 'round': $r, 'stop_after_decide_us': d['stop_after_decide_us'], 'result_ms_p50': d['result_ms_p50'], 'finish_ms_p50': d['finish_ms_p50'], 'late_nonces_losers': d['late_nonces_losers']['p50']}))" >> $OUT || exit $?
  done
done
cat $OUT
