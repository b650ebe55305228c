set -e
mkdir -p gpurun_out
timeout -k 10 200 python3 -u -m pytest tests/test_gpu_pool.py -x -v --timeout 120 --timeout-method thread -m gpu -k "time_budget" > gpurun_out/r04_loop_budget_test.log 2>&1 &&
timeout -k 10 900 python3 tools/experiments/loop_ab.py run 8 > gpurun_out/r04_ab_loop.jsonl 2> gpurun_out/r04_ab_loop.err
