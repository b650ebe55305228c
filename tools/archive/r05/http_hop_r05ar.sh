#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 python3 tools/experiments/http_hop.py > gpurun_out/r05ar_http_hop_probe.json 2> gpurun_out/r05ar_http_hop_probe.err &&
timeout -k 10 300 python3 bench.py --workload receive --steps 300 > gpurun_out/r05ar_receive.json 2> gpurun_out/r05ar_receive.err &&
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r05ar_bench.json 2> gpurun_out/r05ar_bench.err
rc=$?
cat gpurun_out/r05ar_http_hop_probe.json
exit $rc
