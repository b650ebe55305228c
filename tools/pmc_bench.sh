#!/bin/bash
# PMC passes on one bench.py workload: HBM traffic (FETCH_SIZE, WRITE_SIZE, each in its own pass
# as MI355X_MICROARCH.md prescribes) and issue counters, then tools/pmc_summary.py.
# Usage (on the GPU box): tools/pmc_bench.sh TAG KERNEL_SUBSTR OUT_JSON -- <bench.py args>
# Outputs under gpurun_out/pmc_TAG_{fetch,write,sq}.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TAG=$1; KERN=$2; OUT=$3; shift 4
B="python3 bench.py --no-cpu-baseline --http-requests 0 $*"
D=gpurun_out/pmc_$TAG
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d ${D}_fetch -o run -- $B > ${D}_fetch.log 2>&1 &&
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d ${D}_write -o run -- $B > ${D}_write.log 2>&1 &&
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE --output-format csv -d ${D}_sq -o run -- $B > ${D}_sq.log 2>&1 &&
python3 tools/pmc_summary.py $D "$KERN" "rocprofv3 --pmc on \`python3 bench.py $*\` (tools/pmc_bench.sh), one counter group per pass" $OUT
