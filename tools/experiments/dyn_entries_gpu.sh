# Early finish + dynamic entries: GPU suite, single-search A/B against the round's previous library
# (build/abls/prev), and concurrent-request latency (sustained, depth 4 / 8) for both.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_dyn.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_dyn.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_dyn.log
timeout -k 10 300 python3 tools/experiments/lockstep_ab.py run 3 200 tree prev > gpurun_out/dyn_ab.jsonl || exit 1
for d in 4 8; do
  timeout -k 10 120 python3 bench.py --workload sustained --duration 15 --depth $d > gpurun_out/dsust_tree_d$d.json 2>> gpurun_out/dsust.err || exit 1
  NANOPOW_LIB=$PWD/build/abls/prev/libnanopow.so timeout -k 10 120 python3 bench.py --workload sustained --duration 15 --depth $d > gpurun_out/dsust_prev_d$d.json 2>> gpurun_out/dsust.err || exit 1
done
