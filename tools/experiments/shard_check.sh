# Per-XCD workgroup counters: GPU suite, receive-difficulty latency, serial A/B, PMC traffic.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_$1.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_$1.log; exit 1; }
tail -n 1 gpurun_out/pytest_gpu_$1.log
timeout -k 10 300 python3 bench.py --workload receive --steps 200 > gpurun_out/receive_$1.json 2> gpurun_out/receive_$1.err || exit 1
NANOPOW_LIB=$PWD/build/abls/prev/libnanopow.so timeout -k 10 300 python3 bench.py --workload receive --steps 200 > gpurun_out/receive_prev_$1.json 2>> gpurun_out/receive_$1.err || exit 1
bash tools/experiments/pmc_quick.sh $1
