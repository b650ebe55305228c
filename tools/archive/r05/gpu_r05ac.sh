#!/bin/bash
# Round 5, session ac: which change gave the 8-partition overshoot its multi-ms tail -- the overshoot worker over 8
# partitions with the libraries of 79481b0 (per-workgroup fence), 2addcf9 (one per XCD) and the tree (polls past the
# caches), twice each.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r05ac}
O="python3 tests/overshoot_worker.py 200 receive"
for r in 1 2; do
  for L in 79481b0 2addcf9 tree; do
    if [ $L = tree ]; then unset NANOPOW_LIB; else export NANOPOW_LIB=$PWD/build/lib_$L/libnanopow.so; fi
    NANOPOW_TEST_HOOKS=1 NANOPOW_VIRTUAL_DEVICES=8 timeout -k 10 120 $O > gpurun_out/${T}_${L}_$r.json 2> gpurun_out/${T}_${L}_$r.err || exit 1
    echo "$L $r $(grep -o '"stop_after_decide_us": {[^}]*}' gpurun_out/${T}_${L}_$r.json)"
  done
done
