#!/bin/bash
# Round 5, session b: where the 8-partition stop span goes (overshoot worker and the regime with the pool workers'
# step timing and per-search stop timelines), the GPU suite on the fixed tests, the kernel A/B r04 vs tree.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r05b}
PYT="python3 -u -m pytest -x -v --timeout 300 --timeout-method thread"
NANOPOW_TEST_HOOKS=1 NANOPOW_TRACE_STEPS=1 NANOPOW_TRACE_LATENCY=1 NANOPOW_VIRTUAL_DEVICES=8 timeout -k 10 200 python3 tests/overshoot_worker.py 200 receive > gpurun_out/${T}_over8.json 2> gpurun_out/${T}_over8.err &&
NANOPOW_TEST_HOOKS=1 NANOPOW_TRACE_STEPS=1 NANOPOW_TRACE_LATENCY=1 NANOPOW_VIRTUAL_DEVICES=4 timeout -k 10 200 python3 tests/overshoot_worker.py 200 receive > gpurun_out/${T}_over4.json 2> gpurun_out/${T}_over4.err &&
NANOPOW_TRACE_STEPS=1 NANOPOW_VIRTUAL_DEVICES=8 timeout -k 10 300 python3 bench.py --workload regime --gpus 8 --steps 1000 --http-requests 0 > gpurun_out/${T}_regime8.json 2> gpurun_out/${T}_regime8.err &&
NANOPOW_VIRTUAL_DEVICES=8 NANOPOW_VIRTUAL_PARTITION=share timeout -k 10 300 python3 bench.py --workload regime --gpus 8 --steps 1000 --http-requests 0 > gpurun_out/${T}_regime8_share.json 2> gpurun_out/${T}_regime8_share.err &&
timeout -k 10 900 $PYT tests -m gpu > gpurun_out/${T}_pytest_gpu.log 2>&1 &&
timeout -k 10 600 python3 tools/experiments/lib_arms_ab.py 3 r04=build/r04lib/libnanopow.so tree=tree > gpurun_out/${T}_ab_r04_tree.jsonl 2> gpurun_out/${T}_ab.err
rc=$?
tail -n 3 gpurun_out/${T}_pytest_gpu.log
exit $rc
