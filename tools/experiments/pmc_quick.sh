# PMC traffic of the search kernel on the bench workload + the serial A/B against the round's
# previous library (build/abls/prev), for one build.
set -o pipefail
mkdir -p gpurun_out
bash tools/pmc_bench.sh $1 npow_pool_kernel_ls2 gpurun_out/pmc_pool_$1.json -- --steps 100 --warmup 5 --latency-searches 0 || exit 1
timeout -k 10 400 python3 tools/experiments/lockstep_ab.py run 3 200 tree prev > gpurun_out/ab_$1.jsonl || exit 1
