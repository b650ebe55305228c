#!/bin/bash
# Re-run every bench.py workload of profiles/rNN_bench_workloads.jsonl on the GPU box, one line each,
# into gpurun_out/workloads_TAG.jsonl.  Each step has its own time limit; the chain stops at a failure.
set -o pipefail
TAG=${1:-r02}
OUT=gpurun_out/workloads_$TAG.jsonl
mkdir -p gpurun_out && : > $OUT
B="python3 bench.py --no-cpu-baseline"
timeout -k 10 200 $B --workload sweep >> $OUT 2>gpurun_out/wl_sweep.err &&
timeout -k 10 200 $B --workload burst --roots 512 >> $OUT 2>gpurun_out/wl_burst.err &&
timeout -k 10 200 $B --workload burst --roots 512 --via http >> $OUT 2>gpurun_out/wl_bursthttp.err &&
timeout -k 10 200 $B --workload sustained --duration 60 >> $OUT 2>gpurun_out/wl_sustained.err &&
timeout -k 10 200 $B --workload allgpus --steps 100 >> $OUT 2>gpurun_out/wl_allgpus.err &&
timeout -k 10 200 $B --workload dpow --roots 300 --rate 20 >> $OUT 2>gpurun_out/wl_dpow1.err &&
timeout -k 10 200 $B --workload dpow --roots 300 --rate 20 --concurrency 4 >> $OUT 2>gpurun_out/wl_dpow4.err &&
timeout -k 10 300 python3 bench.py --workload receive --steps 200 >> $OUT 2>gpurun_out/wl_receive.err
