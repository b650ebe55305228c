#!/bin/bash
# Effective clock + issue counters for the library sweep kernel and the bare hash loop, same box.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
PM="GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU"
timeout -k 10 60 $R/build/variants/hash_clock_prod 256 8 10 &&
LIBS=$R/nano-dpow_amd/nanopow/libnanopow.so ROUNDS=2 N=17179869184 timeout -k 10 200 python3 $R/tools/experiments/lib_ab.py &&
timeout -k 10 120 rocprofv3 --pmc $PM --output-format csv -d $R/gpurun_out/pmcL_hc -o run -- $R/build/variants/hash_clock_prod 256 8 5 > /dev/null 2>&1 &&
LIBS=$R/nano-dpow_amd/nanopow/libnanopow.so ROUNDS=1 N=17179869184 timeout -k 10 200 rocprofv3 --pmc $PM --output-format csv -d $R/gpurun_out/pmcL_lib -o run -- python3 $R/tools/experiments/lib_ab.py
