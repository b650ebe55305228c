#!/bin/bash
# Round-6 rehearsal of the driver's round-end GPU commands on the current tree, exactly as the driver runs them:
# smoke, `python -m pytest tests/ -x -q -m gpu`, `python bench.py`.  Each with its own time limit; the chain stops at
# the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r06z}
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 &&
timeout -k 10 800 python -u -m pytest tests/ -x -q -m gpu > gpurun_out/${T}_pytest_gpu.log 2>&1 &&
timeout -k 10 300 python bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err
rc=$?
tail -2 gpurun_out/${T}_smoke.log; tail -3 gpurun_out/${T}_pytest_gpu.log; head -c 300 gpurun_out/${T}_bench.json; echo
exit $rc
