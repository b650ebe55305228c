#!/bin/bash
# Round-5 A/B: the per-XCD elected L2 acquire with L1-bypassing header reads; lingering forced on one device.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-xab}
true &&
NANOPOW_LINGER=1 timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_pool.py > gpurun_out/${T}_pytest_pool_linger1.log 2>&1 &&
bash tools/overshoot_runs.sh ${T}_ovr 3 &&
for L in 1 0 1 0; do
  NANOPOW_LINGER=$L timeout -k 10 200 python3 bench.py --workload receive --steps 300 > gpurun_out/${T}_receive_L$L.json 2> gpurun_out/${T}_receive_L$L.err || exit 1
  echo "receive L$L $(head -c 400 gpurun_out/${T}_receive_L$L.json)"
done &&
timeout -k 10 600 python3 tools/experiments/regime_ab.py 2 1500 w1L=1@NANOPOW_LINGER=1 w1=1@NANOPOW_LINGER=0 w8=8 > gpurun_out/${T}_regime_ab.jsonl 2> gpurun_out/${T}_regime_ab.err
