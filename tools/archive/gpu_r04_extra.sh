#!/bin/bash
# Round-4 closing extras on the final build: the multi-device worker (with the values-on-a-partition check),
# BASELINE configs[3] / [4] over 8 CU partitions with their JSON lines kept, the pool soaks and the workloads.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r04h}
PYT="python3 -u -m pytest -x -v -s --timeout 400 --timeout-method thread"
timeout -k 10 200 $PYT tests/test_gpu_multidevice.py::test_four_logical_devices > gpurun_out/${T}_multidev.log 2>&1 &&
timeout -k 10 500 $PYT tests/test_gpu_configs.py > gpurun_out/${T}_pytest_gpu_configs_3_4.log 2>&1 &&
./tools/soaks_r04.sh $T &&
./tools/workloads_refresh.sh $T &&
if [ "${HWQ:-0}" = 1 ]; then ./tools/experiments/hwq_overshoot.sh; fi
rc=$?
tail -n 3 gpurun_out/${T}_pytest_gpu_configs_3_4.log; exit $rc
