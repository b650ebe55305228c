#!/bin/bash
# Round 5, session v: does the fresh-entry acquire fence (ls2_fresh) hold up the joins of a lingering launch?  The
# diagnostic library with and without it (build/diag, build/diag2) under the regime workload, 1 device and 8 partitions.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r05v}
B="python3 bench.py --workload regime --steps 400 --http-requests 0"
export NANOPOW_TRACE_LATENCY=1
NANOPOW_LIB=$PWD/build/diag/libnanopow.so timeout -k 10 200 $B --gpus 1 > gpurun_out/${T}_f1.json 2> gpurun_out/${T}_f1.err &&
NANOPOW_LIB=$PWD/build/diag2/libnanopow.so timeout -k 10 200 $B --gpus 1 > gpurun_out/${T}_x1.json 2> gpurun_out/${T}_x1.err &&
NANOPOW_VIRTUAL_DEVICES=8 NANOPOW_LIB=$PWD/build/diag/libnanopow.so timeout -k 10 200 $B --gpus 8 > gpurun_out/${T}_f8.json 2> gpurun_out/${T}_f8.err &&
NANOPOW_VIRTUAL_DEVICES=8 NANOPOW_LIB=$PWD/build/diag2/libnanopow.so timeout -k 10 200 $B --gpus 8 > gpurun_out/${T}_x8.json 2> gpurun_out/${T}_x8.err
