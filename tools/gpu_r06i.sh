#!/bin/bash
# Round-6 A/B of the watcher's and waiters' spin window: the job's expected time (new) against a flat 2 ms
# (build/base_r06f), interleaved, on the 8-GPU time regime over 1 GPU and over 8 CU partitions, and on the default
# bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r06i}
R1="python3 bench.py --workload regime --gpus 1 --steps 2000 --http-requests 0"
R8="python3 bench.py --workload regime --gpus 8 --steps 2000 --http-requests 0"
B="python3 bench.py --no-cpu-baseline --steps 100 --warmup 5 --latency-searches 300 --http-requests 0 --regime-searches 0"
L=build/base_r06f/libnanopow.so
for i in 1 2; do
  timeout -k 10 200 $R1 > gpurun_out/${T}_r1_new$i.json 2> gpurun_out/${T}_r1_new$i.err || exit 1
  NANOPOW_LIB=$L timeout -k 10 200 $R1 > gpurun_out/${T}_r1_base$i.json 2> gpurun_out/${T}_r1_base$i.err || exit 1
  NANOPOW_VIRTUAL_DEVICES=8 timeout -k 10 200 $R8 > gpurun_out/${T}_r8_new$i.json 2> gpurun_out/${T}_r8_new$i.err || exit 1
  NANOPOW_VIRTUAL_DEVICES=8 NANOPOW_LIB=$L timeout -k 10 200 $R8 > gpurun_out/${T}_r8_base$i.json 2> gpurun_out/${T}_r8_base$i.err || exit 1
done
timeout -k 10 150 $B > gpurun_out/${T}_b_new.json 2> gpurun_out/${T}_b_new.err &&
NANOPOW_LIB=$L timeout -k 10 150 $B > gpurun_out/${T}_b_base.json 2> gpurun_out/${T}_b_base.err
rc=$?
for f in gpurun_out/${T}_r*.json gpurun_out/${T}_b_*.json; do python3 -c "
import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); r=d.get('node_ttw_8x_regime') or {}
print('$f'.split('/')[-1], d.get('value'), r.get('node_over_kernel'), r.get('node_over_reference'), (r.get('fixed_cost_us') or {}).get('fixed_us'), r.get('p50_minus_expected_ms'), (d.get('ttw_c_abi_ms') or {}).get('p50'))"; done
exit $rc
