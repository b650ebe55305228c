#!/bin/bash
# Round 3, final shape (four 512-lane workgroups per CU): stream variants against the shipped one --
# priority 2 for alignbits / 1 for adds, adds after alignbits in each half-rate run, the odd placement.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 tools/experiments/setprio_ab.py run 4 150 tree pad_ad sp_order pad_o128 > gpurun_out/r03_ab_stream_w8.jsonl 2> gpurun_out/r03_ab_stream_w8.err
rc=$?
cat gpurun_out/r03_ab_stream_w8.jsonl; tail -3 gpurun_out/r03_ab_stream_w8.err
exit $rc
