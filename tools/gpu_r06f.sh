#!/bin/bash
# Round-6 closing GPU session, part 1 (the driver's own commands on the final tree): smoke, the whole GPU suite as the
# driver runs it (-x, ordered: parity and server first), the bench with no flags and with --steps 20 --warmup 5.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r06f}
timeout -k 10 180 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 &&
timeout -k 10 800 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1 &&
timeout -k 10 300 python3 bench.py > gpurun_out/${T}_bench_noflags.json 2> gpurun_out/${T}_bench_noflags.err &&
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err
rc=$?
tail -3 gpurun_out/${T}_smoke.log; tail -3 gpurun_out/${T}_pytest_gpu.log
head -c 600 gpurun_out/${T}_bench_noflags.json; echo; head -c 400 gpurun_out/${T}_bench.json; echo
exit $rc
