#!/bin/bash
# Round 5: lingering on / off by partition size (2 / 4 / 8 CU partitions and the whole GPU) on the final build -- the
# 2^26 regime interleaved, then the first-found stop span over 4 and 8 partitions with lingering off.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-lda}
timeout -k 10 900 python3 tools/experiments/regime_ab.py 2 1500 l1=1@NANOPOW_LINGER=1 n1=1@NANOPOW_LINGER=0 l2=2@NANOPOW_LINGER=1 n2=2@NANOPOW_LINGER=0 l4=4@NANOPOW_LINGER=1 n4=4@NANOPOW_LINGER=0 l8=8@NANOPOW_LINGER=1 n8=8@NANOPOW_LINGER=0 > gpurun_out/${T}_regime_ab.jsonl 2> gpurun_out/${T}_regime_ab.err || exit 1
for r in 1 2 3; do
  for g in 4 8; do
    for L in 0 1; do
      NANOPOW_LINGER=$L NANOPOW_TEST_HOOKS=1 NANOPOW_VIRTUAL_DEVICES=$g timeout -k 10 120 python3 tests/overshoot_worker.py 200 receive > gpurun_out/${T}_ovr_g${g}_L${L}_$r.json 2> gpurun_out/${T}_ovr_g${g}_L${L}_$r.err || exit 1
      echo "g$g L$L $r $(grep -o '"stop_after_decide_us": {[^}]*}' gpurun_out/${T}_ovr_g${g}_L${L}_$r.json)"
    done
  done
done
