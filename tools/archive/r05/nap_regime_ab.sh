#!/bin/bash
# Round 5: the pool worker's nap between steps (NANOPOW_POLL_US, 50 us) re-measured at the 2^26
# regime's time scale, on the whole GPU and over 8 CU partitions, interleaved.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-nap}
timeout -k 10 900 python3 tools/experiments/regime_ab.py 2 1500 n50w1=1@NANOPOW_POLL_US=50 n20w1=1@NANOPOW_POLL_US=20 n0w1=1@NANOPOW_POLL_US=0 n50w8=8@NANOPOW_POLL_US=50 n20w8=8@NANOPOW_POLL_US=20 n0w8=8@NANOPOW_POLL_US=0 > gpurun_out/${T}_regime_ab.jsonl 2> gpurun_out/${T}_regime_ab.err
