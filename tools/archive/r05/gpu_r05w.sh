#!/bin/bash
# Round 5, session w: every workgroup's entry start after a published dynamic entry (diagnostic library), serial
# searches waited to the end, one device, lingering on; the regime workload the same way.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r05w}
export NANOPOW_LIB=$PWD/build/diag/libnanopow.so
LAT_STDERR=gpurun_out/${T}_serial.err timeout -k 10 200 python3 tools/experiments/lat_fields.py 200 ffffffc000000000 > gpurun_out/${T}_serial.json 2>&1 &&
NANOPOW_TRACE_LATENCY=1 timeout -k 10 200 python3 bench.py --workload regime --steps 200 --http-requests 0 --gpus 1 > gpurun_out/${T}_regime.json 2> gpurun_out/${T}_regime.err
