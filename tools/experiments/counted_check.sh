# Counting only in launches of 2+ entries: GPU suite, fixed per-search overhead and receive latency
# (latency_probe) and serial A/B against build/abls/prev, closed-loop sustained at depth 4 for both.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_cnt.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_cnt.log; exit 1; }
tail -n 1 gpurun_out/pytest_gpu_cnt.log
for arm in tree prev; do
  L=$PWD/nano-dpow_amd/nanopow/libnanopow.so; [ $arm = prev ] && L=$PWD/build/abls/prev/libnanopow.so
  NANOPOW_LIB=$L timeout -k 10 120 python3 tools/latency_probe.py 300 > gpurun_out/latc_$arm.json || exit 1
  NANOPOW_LIB=$L timeout -k 10 120 python3 bench.py --workload sustained --duration 15 --depth 4 > gpurun_out/sustc_$arm.json 2>> gpurun_out/sustc.err || exit 1
done
timeout -k 10 400 python3 tools/experiments/lockstep_ab.py run 3 200 tree prev > gpurun_out/ab_cnt.jsonl || exit 1
cat gpurun_out/latc_tree.json gpurun_out/latc_prev.json
