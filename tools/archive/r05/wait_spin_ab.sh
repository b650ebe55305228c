#!/bin/bash
# Round 5: result waits that poll before sleeping (npow_wait_result, NANOPOW_WAIT_SPIN) -- the regime on the whole GPU
# and over 8 CU partitions, and the receive workload, interleaved on and off.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-wsp}
timeout -k 10 900 python3 tools/experiments/regime_ab.py 2 1500 s1=1@NANOPOW_WAIT_SPIN=1 n1=1@NANOPOW_WAIT_SPIN=0 s8=8@NANOPOW_WAIT_SPIN=1 n8=8@NANOPOW_WAIT_SPIN=0 > gpurun_out/${T}_regime_ab.jsonl 2> gpurun_out/${T}_regime_ab.err || exit 1
for S in 1 0 1 0; do
  NANOPOW_WAIT_SPIN=$S timeout -k 10 200 python3 bench.py --workload receive --steps 300 > gpurun_out/${T}_receive_S$S.json 2> gpurun_out/${T}_receive_S$S.err || exit 1
  echo "receive S$S $(python3 -c "import json,sys; r=json.loads(open('gpurun_out/${T}_receive_S$S.json').read().strip().splitlines()[-1])['receive']; print(r['gpu_c_abi_ms']['p50'], r['gpu_http_keepalive_ms']['p50'])")"
done
