#!/bin/bash
# Round 5, first session: smoke; the 8-GPU time regime (one root at a time at ffffffc0 over 8 CU
# partitions) with the new library, the round-4 library and the new one with spinning workers, then 4 partitions
# and the whole GPU; the GPU suite on the new build; the kernel A/B round-4 library vs the new one.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r05a}
PYT="python3 -u -m pytest -x -v --timeout 300 --timeout-method thread"
R="python3 bench.py --workload regime --steps 1000 --http-requests 200"
timeout -k 10 180 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 &&
NANOPOW_VIRTUAL_DEVICES=8 timeout -k 10 300 $R --gpus 8 > gpurun_out/${T}_regime8_new.json 2> gpurun_out/${T}_regime8_new.err &&
NANOPOW_LIB=build/r04lib/libnanopow.so NANOPOW_VIRTUAL_DEVICES=8 timeout -k 10 300 $R --gpus 8 > gpurun_out/${T}_regime8_r04.json 2> gpurun_out/${T}_regime8_r04.err &&
NANOPOW_POLL_US=0 NANOPOW_VIRTUAL_DEVICES=8 timeout -k 10 300 $R --gpus 8 > gpurun_out/${T}_regime8_spin.json 2> gpurun_out/${T}_regime8_spin.err &&
NANOPOW_VIRTUAL_DEVICES=4 timeout -k 10 300 $R --gpus 4 > gpurun_out/${T}_regime4_new.json 2> gpurun_out/${T}_regime4_new.err &&
timeout -k 10 300 $R > gpurun_out/${T}_regime1_new.json 2> gpurun_out/${T}_regime1_new.err &&
timeout -k 10 900 $PYT tests -m gpu > gpurun_out/${T}_pytest_gpu.log 2>&1 &&
timeout -k 10 600 python3 tools/experiments/lib_arms_ab.py 3 r04=build/r04lib/libnanopow.so tree=tree > gpurun_out/${T}_ab_r04_tree.jsonl 2> gpurun_out/${T}_ab.err
rc=$?
tail -n 3 gpurun_out/${T}_pytest_gpu.log
exit $rc
