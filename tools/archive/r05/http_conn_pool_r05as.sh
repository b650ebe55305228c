#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_server.py tests/test_gpu_configs.py > gpurun_out/r05as_pytest.log 2>&1 &&
timeout -k 10 300 python3 bench.py --workload receive --steps 300 > gpurun_out/r05as_receive.json 2> gpurun_out/r05as_receive.err
rc=$?; tail -1 gpurun_out/r05as_pytest.log; exit $rc
