#!/bin/bash
# Round 5, session z: one L2 invalidation per XCD -- regime A/B lingering on/off over 1 / 8 devices, the bench A/B.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r05z}
timeout -k 10 700 python3 tools/experiments/regime_ab.py 2 1000 l1=1 n1=1@NANOPOW_LINGER=0 l8=8 n8=8@NANOPOW_LINGER=0 > gpurun_out/${T}_regime_ab.jsonl 2> gpurun_out/${T}_regime_ab.err &&
timeout -k 10 600 python3 tools/experiments/lib_arms_ab.py 2 tree=tree nl=tree@NANOPOW_LINGER=0 > gpurun_out/${T}_ab.jsonl 2> gpurun_out/${T}_ab.err
rc=$?
cat gpurun_out/${T}_ab.jsonl
exit $rc
