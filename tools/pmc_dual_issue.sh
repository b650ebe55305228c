#!/bin/bash
# VALU dual issue in the search kernel: SQ_ACTIVE_INST_VALU2 ("quad-cycles two VALU instructions are
# issued", per SIMD) beside the VALU totals, one PMC pass over a short bench run.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
D=gpurun_out/pmc_dual${1:+_$1}
timeout -s KILL 150 rocprofv3 --pmc SQ_ACTIVE_INST_VALU2 SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_THREAD_CYCLES_VALU SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d $D -o run -- python3 bench.py --no-cpu-baseline --steps 30 --warmup 3 --latency-searches 0 --http-requests 0 --regime-searches 0 > ${D}.log 2>&1
rc=$?
ls $D; exit $rc
