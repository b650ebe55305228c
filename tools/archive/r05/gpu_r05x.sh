#!/bin/bash
# Round 5, session x: the lingering workgroups' pinned-read period (NANOPOW_LINGER_P) against their join spread
# (diagnostic library, serial searches, one device).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r05x}
export NANOPOW_LIB=$PWD/build/diag/libnanopow.so
for P in 512 64 8 1; do
  NANOPOW_LINGER_P=$P LAT_STDERR=gpurun_out/${T}_p$P.err timeout -k 10 200 python3 tools/experiments/lat_fields.py 150 ffffffc000000000 > gpurun_out/${T}_p$P.json 2>&1 || exit 1
done
