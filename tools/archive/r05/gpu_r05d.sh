#!/bin/bash
# Round 5, session d: (1) is the 8-CU-partition stop tail the number of hardware queues? 4 partitions with 4 idle extra
# CU-masked queues, 8 partitions with 4 of them searching (0x55), and 8 partitions (baseline); (2) the regime
# interleaved, watcher on / off, over 1 / 4 / 8 devices; (3) the driver's bench command.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r05d}
O="timeout -k 10 200 python3 tests/overshoot_worker.py 200 receive"
NANOPOW_TEST_HOOKS=1 NANOPOW_VIRTUAL_DEVICES=4 NANOPOW_TEST_EXTRA_QUEUES=4 $O > gpurun_out/${T}_over_g4_q4.json 2> gpurun_out/${T}_over_g4_q4.err &&
NANOPOW_TEST_HOOKS=1 NANOPOW_VIRTUAL_DEVICES=4 NANOPOW_TEST_EXTRA_QUEUES=1 $O > gpurun_out/${T}_over_g4_q1.json 2> gpurun_out/${T}_over_g4_q1.err &&
NANOPOW_TEST_HOOKS=1 NANOPOW_VIRTUAL_DEVICES=4 $O > gpurun_out/${T}_over_g4.json 2> gpurun_out/${T}_over_g4.err &&
NANOPOW_TEST_HOOKS=1 NANOPOW_VIRTUAL_DEVICES=8 $O 0x55 > gpurun_out/${T}_over_g8_m55.json 2> gpurun_out/${T}_over_g8_m55.err &&
NANOPOW_TEST_HOOKS=1 NANOPOW_VIRTUAL_DEVICES=8 $O > gpurun_out/${T}_over_g8.json 2> gpurun_out/${T}_over_g8.err &&
timeout -k 10 600 python3 tools/experiments/regime_ab.py 2 1000 w1=1 nw1=1@NANOPOW_WATCHER=0 w4=4 nw4=4@NANOPOW_WATCHER=0 w8=8 nw8=8@NANOPOW_WATCHER=0 > gpurun_out/${T}_regime_ab.jsonl 2> gpurun_out/${T}_regime_ab.err &&
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err
rc=$?
head -c 600 gpurun_out/${T}_bench.json
exit $rc
