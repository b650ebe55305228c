#!/bin/bash
# Round 5, session g: the poll schedule spread over the grid -- GPU timelines of the kill relay (diagnostic build) on
# 8 / 4 partitions, the overshoot worker on the shipped build (8, 4, and 8 with 4 searching), the kernel A/B
# against the round-4 library (one more SALU op per iteration), the regime on 8.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r05g}
O="timeout -k 10 200 python3 tests/overshoot_worker.py"
NANOPOW_LIB=build/diag/libnanopow.so NANOPOW_TRACE_LATENCY=1 NANOPOW_VIRTUAL_DEVICES=8 $O 100 receive > gpurun_out/${T}_diag_g8.json 2> gpurun_out/${T}_diag_g8.err &&
NANOPOW_LIB=build/diag/libnanopow.so NANOPOW_TRACE_LATENCY=1 NANOPOW_VIRTUAL_DEVICES=4 $O 100 receive > gpurun_out/${T}_diag_g4.json 2> gpurun_out/${T}_diag_g4.err &&
NANOPOW_TEST_HOOKS=1 NANOPOW_VIRTUAL_DEVICES=8 $O 200 receive > gpurun_out/${T}_over_g8.json 2> gpurun_out/${T}_over_g8.err &&
NANOPOW_TEST_HOOKS=1 NANOPOW_VIRTUAL_DEVICES=4 $O 200 receive > gpurun_out/${T}_over_g4.json 2> gpurun_out/${T}_over_g4.err &&
NANOPOW_TEST_HOOKS=1 NANOPOW_VIRTUAL_DEVICES=8 $O 200 receive 0x55 > gpurun_out/${T}_over_g8_m55.json 2> gpurun_out/${T}_over_g8_m55.err &&
NANOPOW_VIRTUAL_DEVICES=8 timeout -k 10 300 python3 bench.py --workload regime --gpus 8 --steps 1000 --http-requests 200 > gpurun_out/${T}_regime8.json 2> gpurun_out/${T}_regime8.err &&
timeout -k 10 600 python3 tools/experiments/lib_arms_ab.py 3 r04=build/r04lib/libnanopow.so tree=tree > gpurun_out/${T}_ab_r04_tree.jsonl 2> gpurun_out/${T}_ab.err
