#!/bin/bash
# Round 5, session p: how long a yielded lingering launch takes to end, over 8 CU partitions and on the whole GPU.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r05p}
NANOPOW_DEBUG=1 NANOPOW_VIRTUAL_DEVICES=8 timeout -k 10 120 python3 tools/experiments/linger_probe.py 3 70 > gpurun_out/${T}_probe8.txt 2> gpurun_out/${T}_probe8.err &&
NANOPOW_DEBUG=1 timeout -k 10 120 python3 tools/experiments/linger_probe.py 3 70 > gpurun_out/${T}_probe1.txt 2> gpurun_out/${T}_probe1.err
rc=$?
cat gpurun_out/${T}_probe8.txt gpurun_out/${T}_probe1.txt
exit $rc
