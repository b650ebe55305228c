#!/bin/bash
# Round 5: lingering on / off over 8 CU partitions (the only size where it is on by default), 4 interleaved rounds of
# 2,000 searches each -- the default's evidence with more samples.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python3 tools/experiments/regime_ab.py 4 2000 l8=8@NANOPOW_LINGER=1 n8=8@NANOPOW_LINGER=0 > gpurun_out/r05aw_linger8_regime_ab.jsonl 2> gpurun_out/r05aw_linger8_regime_ab.err
