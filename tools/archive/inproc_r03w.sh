#!/bin/bash
# Round-3 final build: bench.py --gpus N in one process (the product's multi-device pool) over 2 and 8
# logical devices on the one GPU, with node time-to-work and overshoot per search.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
NANOPOW_VIRTUAL_DEVICES=2 timeout -k 10 300 python3 bench.py --gpus 2 --steps 60 --warmup 4 --node-searches 100 > gpurun_out/r03w_bench_inproc_2vd.json 2> gpurun_out/r03w_bench_inproc_2vd.err &&
NANOPOW_VIRTUAL_DEVICES=8 timeout -k 10 300 python3 bench.py --gpus 8 --steps 15 --warmup 2 --node-searches 100 > gpurun_out/r03w_bench_inproc_8vd.json 2> gpurun_out/r03w_bench_inproc_8vd.err
rc=$?
head -c 600 gpurun_out/r03w_bench_inproc_2vd.json; echo; head -c 600 gpurun_out/r03w_bench_inproc_8vd.json; echo
exit $rc
