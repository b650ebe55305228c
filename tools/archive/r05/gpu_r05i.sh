#!/bin/bash
# Round 5, session i: where the 8-partition regime's kernel time goes -- per-launch event span against the clock
# waves' span (tools/experiments/launch_spans.py) over 8 partitions and 1 device, then the regime A/B with the host-word
# poll interval scaled to the partition's size (NANOPOW_POLL=128: the whole GPU's 8 polls per iteration on each
# 32-CU partition) and with 8 hardware queues.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r05i}
L="python3 tools/experiments/launch_spans.py"
timeout -k 10 200 $L 8 400 > gpurun_out/${T}_spans.jsonl 2> gpurun_out/${T}_spans.err &&
timeout -k 10 200 $L 1 400 >> gpurun_out/${T}_spans.jsonl 2>> gpurun_out/${T}_spans.err &&
timeout -k 10 200 $L 8 400 NANOPOW_POLL=128 >> gpurun_out/${T}_spans.jsonl 2>> gpurun_out/${T}_spans.err &&
timeout -k 10 200 $L 8 400 GPU_MAX_HW_QUEUES=8 >> gpurun_out/${T}_spans.jsonl 2>> gpurun_out/${T}_spans.err &&
timeout -k 10 600 python3 tools/experiments/regime_ab.py 2 1000 n8=8 p8=8@NANOPOW_POLL=128 q8=8@GPU_MAX_HW_QUEUES=8 > gpurun_out/${T}_regime_ab.jsonl 2> gpurun_out/${T}_regime_ab.err
rc=$?
cat gpurun_out/${T}_spans.jsonl
exit $rc
