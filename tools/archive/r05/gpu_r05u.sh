#!/bin/bash
# Round 5, session u: the diagnostic library's join / win timestamps under the regime workload, one device and 8 CU
# partitions, lingering on and off (the gap between one search's win and the next one's hashing).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r05u}
B="python3 bench.py --workload regime --steps 400 --http-requests 0"
export NANOPOW_LIB=$PWD/build/diag/libnanopow.so NANOPOW_TRACE_LATENCY=1
timeout -k 10 200 $B --gpus 1 > gpurun_out/${T}_l1.json 2> gpurun_out/${T}_l1.err &&
NANOPOW_LINGER=0 timeout -k 10 200 $B --gpus 1 > gpurun_out/${T}_n1.json 2> gpurun_out/${T}_n1.err &&
NANOPOW_VIRTUAL_DEVICES=8 timeout -k 10 200 $B --gpus 8 > gpurun_out/${T}_l8.json 2> gpurun_out/${T}_l8.err &&
NANOPOW_VIRTUAL_DEVICES=8 NANOPOW_LINGER=0 timeout -k 10 200 $B --gpus 8 > gpurun_out/${T}_n8.json 2> gpurun_out/${T}_n8.err
