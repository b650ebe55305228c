#!/bin/bash
# PMC passes on the bench workload (npow_pool_kernel): HBM traffic (FETCH_SIZE, WRITE_SIZE, each in
# its own pass as MI355X_MICROARCH.md prescribes) and issue counters.  Outputs under gpurun_out/pmc_*.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
B="python3 bench.py --no-cpu-baseline --steps 40 --warmup 2"
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o run -- $B > gpurun_out/pmc_fetch.log 2>&1 &&
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o run -- $B > gpurun_out/pmc_write.log 2>&1 &&
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc_sq -o run -- $B > gpurun_out/pmc_sq.log 2>&1
