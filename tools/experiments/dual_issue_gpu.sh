#!/bin/bash
# GPU box: the dual-issue probe alone (instructions per SIMD-cycle per class pair) and under one PMC
# pass (SQ_ACTIVE_INST_VALU2 per kernel).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
S=${1:-half}
timeout -k 10 60 build/dual_issue_$S 20000 > gpurun_out/dual_issue_$S.jsonl 2> gpurun_out/dual_issue_$S.err &&
timeout -s KILL 90 rocprofv3 --pmc SQ_ACTIVE_INST_VALU2 SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc_dual_probe_$S -o run -- build/dual_issue_$S 20000 > gpurun_out/dual_issue_pmc_$S.log 2>&1
rc=$?; cat gpurun_out/dual_issue_$S.jsonl; exit $rc
