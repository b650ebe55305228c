#!/bin/bash
# Round 5: the round-end driver's own commands on a fresh box -- the GPU suite as it invokes it, smoke(), the bench
# with no flags -- each under its own time limit.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -m pytest tests/ -x -q -m gpu > gpurun_out/r05ax_driver_pytest.log 2>&1 &&
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05ax_driver_smoke.log 2>&1 &&
timeout -k 10 400 python bench.py > gpurun_out/r05ax_driver_bench.json 2> gpurun_out/r05ax_driver_bench.err
rc=$?
tail -1 gpurun_out/r05ax_driver_pytest.log; tail -1 gpurun_out/r05ax_driver_smoke.log | cut -c1-100; head -c 300 gpurun_out/r05ax_driver_bench.json
exit $rc
