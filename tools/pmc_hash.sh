#!/bin/bash
# PMC passes over hash_clock variants (no trace domains combined with --pmc).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVES"
P2="SQ_IFETCH SQ_IFETCH_LEVEL SQ_LEVEL_WAVES SQ_INSTS_SALU SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_THREAD_CYCLES_VALU SQ_CYCLES"
for v in "$@"; do
  for p in 1 2; do
    eval PM=\$P$p
    timeout -k 10 120 rocprofv3 --pmc $PM --output-format csv -d $R/gpurun_out/pmc_${v}_$p -o run -- $R/build/variants/hash_clock_$v 256 8 3 > $R/gpurun_out/pmc_${v}_$p.log 2>&1 || exit 1
  done
done
