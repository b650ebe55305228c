#!/bin/bash
# Round 5: which stops come without a published final count under lingering launches (4 CU partitions, lingering
# forced on) -- NANOPOW_TRACE_LATENCY's nanopow-nofin lines beside NANOPOW_DEBUG's launch trace.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-nft}
for r in 1 2 3 4 5 6; do
  NANOPOW_LINGER=1 NANOPOW_TRACE_LATENCY=1 NANOPOW_DEBUG=1 NANOPOW_VIRTUAL_DEVICES=4 timeout -k 10 150 python3 tests/overshoot_worker.py 200 receive > gpurun_out/${T}_g4_$r.json 2> gpurun_out/${T}_g4_$r.err || exit 1
  echo "g4 $r $(grep -o '"stop_after_decide_us": {[^}]*}' gpurun_out/${T}_g4_$r.json) nofin $(grep -c nanopow-nofin gpurun_out/${T}_g4_$r.err)"
done
