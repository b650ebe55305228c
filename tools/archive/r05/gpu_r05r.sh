#!/bin/bash
# Round 5, session r: lingering launches measured -- the bench / receive A/B (pre-lingering library, the tree, the tree
# with NANOPOW_LINGER=0) and the regime A/B over 1 / 4 / 8 devices, lingering on and off.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r05r}
timeout -k 10 600 python3 tools/experiments/lib_arms_ab.py 3 pre=build/r05pre/libnanopow.so tree=tree nl=tree@NANOPOW_LINGER=0 > gpurun_out/${T}_ab.jsonl 2> gpurun_out/${T}_ab.err &&
timeout -k 10 700 python3 tools/experiments/regime_ab.py 2 1000 l1=1 n1=1@NANOPOW_LINGER=0 l4=4 n4=4@NANOPOW_LINGER=0 l8=8 n8=8@NANOPOW_LINGER=0 > gpurun_out/${T}_regime_ab.jsonl 2> gpurun_out/${T}_regime_ab.err
rc=$?
cat gpurun_out/${T}_ab.jsonl
exit $rc
