#!/bin/bash
# Round 5: a draining slot without its final count no longer holds a lingering launch past g_linger_us -- the
# first-found stop span over 4 CU partitions with lingering forced on (where a 21-ms stop was seen) and over 8 (the
# default), then the closing session of this build (tools/close_r05g.sh).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-sdc}
for r in 1 2 3 4 5 6 7 8; do
  for g in 4 8; do
    NANOPOW_LINGER=1 NANOPOW_TEST_HOOKS=1 NANOPOW_VIRTUAL_DEVICES=$g timeout -k 10 120 python3 tests/overshoot_worker.py 200 receive > gpurun_out/${T}_ovr_g${g}_$r.json 2> gpurun_out/${T}_ovr_g${g}_$r.err || exit 1
    echo "g$g $r $(grep -o '"stop_after_decide_us": {[^}]*}' gpurun_out/${T}_ovr_g${g}_$r.json)"
  done
done
bash tools/close_r05g.sh $T
