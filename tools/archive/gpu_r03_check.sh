set -o pipefail
export TMPDIR=/tmp
PYT="python3 -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 300 $PYT -s tests/test_gpu_multidevice.py tests/test_gpu_pool.py > gpurun_out/r03g_pytest.log 2>&1 &&
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r03g_bench.json 2> gpurun_out/r03g_bench.err
rc=$?; tail -2 gpurun_out/r03g_pytest.log; grep overshoot gpurun_out/r03g_pytest.log | cut -c1-300; exit $rc
