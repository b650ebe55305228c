set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_early.log 2>&1 &&
timeout -k 10 300 python3 tools/experiments/lockstep_ab.py run 3 200 tree prev sp_ad > gpurun_out/early_ab.jsonl &&
timeout -k 10 120 python3 bench.py --workload sustained --duration 20 --depth 4 > gpurun_out/sust_tree.json 2> gpurun_out/sust_tree.err &&
NANOPOW_LIB=$PWD/build/abls/prev/libnanopow.so timeout -k 10 120 python3 bench.py --workload sustained --duration 20 --depth 4 > gpurun_out/sust_prev.json 2> gpurun_out/sust_prev.err
rc=$?
tail -3 gpurun_out/pytest_gpu_early.log
exit $rc
