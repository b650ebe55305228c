#!/bin/bash
# Round 5, session y: the XCC id probe, then the join spread with one L2 invalidation per XCD (diagnostic library),
# then the linger tests.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r05y}
timeout -k 5 60 ./build/xcc_probe > gpurun_out/${T}_xcc.txt 2>&1 &&
NANOPOW_LIB=$PWD/build/diag/libnanopow.so LAT_STDERR=gpurun_out/${T}_serial.err timeout -k 10 120 python3 tools/experiments/lat_fields.py 150 ffffffc000000000 > gpurun_out/${T}_serial.json 2>&1 &&
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_linger.py > gpurun_out/${T}_linger.log 2>&1
rc=$?
cat gpurun_out/${T}_xcc.txt; tail -n 2 gpurun_out/${T}_linger.log
exit $rc
