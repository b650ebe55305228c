#!/bin/bash
# Round-4 A/Bs: where the search loop acts on a stop request (tools/experiments/stop_ab.py), and
# energy per hash of 8 / 6 / 4 waves per SIMD (tools/experiments/energy_ab.py).  Each step has its own
# time limit; the chain stops at the first failure.
set -o pipefail
TAG=${1:-r04}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python3 tools/experiments/stop_ab.py run 2 > gpurun_out/${TAG}_ab_stop.jsonl 2> gpurun_out/${TAG}_ab_stop.err &&
timeout -k 10 400 python3 tools/experiments/energy_ab.py run 3 150 g4 g3 g2 > gpurun_out/${TAG}_ab_energy.jsonl 2> gpurun_out/${TAG}_ab_energy.err
rc=$?
cat gpurun_out/${TAG}_ab_stop.jsonl gpurun_out/${TAG}_ab_energy.jsonl; tail -3 gpurun_out/${TAG}_ab_stop.err gpurun_out/${TAG}_ab_energy.err
exit $rc
