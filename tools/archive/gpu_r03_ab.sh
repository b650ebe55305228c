#!/bin/bash
# Round-3 GPU session 2: the static s_setprio A/B, the in-process --gpus path rehearsed over logical
# devices, and the --gpus check against the visible devices.  Each GPU step has its own time limit.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 420 python3 tools/experiments/setprio_ab.py run 4 200 base prio1 prio2 prio3 > gpurun_out/r03_ab_setprio.jsonl 2> gpurun_out/r03_ab_setprio.err &&
NANOPOW_VIRTUAL_DEVICES=2 timeout -k 10 300 python3 bench.py --gpus 2 --steps 60 --warmup 4 --node-searches 100 > gpurun_out/r03_bench_inproc_2vd.json 2> gpurun_out/r03_bench_inproc_2vd.err &&
NANOPOW_VIRTUAL_DEVICES=8 timeout -k 10 300 python3 bench.py --gpus 8 --steps 15 --warmup 2 --node-searches 100 > gpurun_out/r03_bench_inproc_8vd.json 2> gpurun_out/r03_bench_inproc_8vd.err
rc=$?
( timeout -k 10 120 python3 bench.py --gpus 2 --steps 2 --warmup 0 --no-cpu-baseline > gpurun_out/r03_bench_gpus2_on_1gpu.out 2>&1; echo "exit=$?" >> gpurun_out/r03_bench_gpus2_on_1gpu.out )
cat gpurun_out/r03_ab_setprio.jsonl; head -c 1500 gpurun_out/r03_bench_inproc_2vd.json; tail -2 gpurun_out/r03_bench_gpus2_on_1gpu.out
exit $rc
