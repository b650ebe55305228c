# Concurrent-request latency with and without early finish (in-tree library vs build/abls/prev):
# bench.py --workload sustained at depth 4 and 8, two interleaved rounds.
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
  for d in 4 8; do
    timeout -k 10 120 python3 bench.py --workload sustained --duration 15 --depth $d > gpurun_out/sust_tree_d${d}_r$r.json 2>> gpurun_out/sust.err || exit 1
    NANOPOW_LIB=$PWD/build/abls/prev/libnanopow.so timeout -k 10 120 python3 bench.py --workload sustained --duration 15 --depth $d > gpurun_out/sust_prev_d${d}_r$r.json 2>> gpurun_out/sust.err || exit 1
  done
done
