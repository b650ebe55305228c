set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
NANOPOW_VIRTUAL_DEVICES=8 NANOPOW_TRACE_LATENCY=1 timeout -k 10 120 python3 tests/overshoot_worker.py 100 receive > gpurun_out/r04c_os8.json 2> gpurun_out/r04c_os8.trace &&
NANOPOW_VIRTUAL_DEVICES=4 NANOPOW_TRACE_LATENCY=1 timeout -k 10 120 python3 tests/overshoot_worker.py 100 receive > gpurun_out/r04c_os4.json 2> gpurun_out/r04c_os4.trace &&
./tools/gpu_r04.sh r04c
