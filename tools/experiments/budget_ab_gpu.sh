set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_dyn2.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_dyn2.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_dyn2.log
timeout -k 10 500 python3 tools/experiments/lockstep_ab.py run 4 200 tree prev NANOPOW_BUDGET_US=40000 > gpurun_out/ab4.jsonl || exit 1
# pool soaks on the early-finish / dynamic-entry build: one device, 4 logical devices, and 4 logical
# devices with device 1's wins corrupted (dropped after 3)
timeout -k 10 150 python3 -u tools/pool_soak.py --seconds 60 > gpurun_out/soak_dyn.log 2>&1 || exit 1
NANOPOW_VIRTUAL_DEVICES=4 timeout -k 10 150 python3 -u tools/pool_soak.py --seconds 60 > gpurun_out/soak_dyn_4vd.log 2>&1 || exit 1
NANOPOW_VIRTUAL_DEVICES=4 NANOPOW_FAULT_INVALID=1 timeout -k 10 150 python3 -u tools/pool_soak.py --seconds 60 --faults > gpurun_out/soak_dyn_fault.log 2>&1 || exit 1
tail -n 1 gpurun_out/soak_dyn.log gpurun_out/soak_dyn_4vd.log gpurun_out/soak_dyn_fault.log
