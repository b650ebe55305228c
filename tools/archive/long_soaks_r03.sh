#!/bin/bash
# Round 3, final build: long pool soaks (tools/pool_soak.py, 24 client threads, every result checked):
# 9 minutes on the one device, 260 s over 8 logical devices, 260 s of the UBSan host build over
# 4 logical devices (the whole chain fits one 1,200-s gpurun call; the first run of this script asked
# for 600 + 300 + 300 s and the call limit cut the UBSan soak at 290 s).  Each step has its own time
# limit; the chain stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
LIBDIR=$PWD/nano-dpow_amd/nanopow
timeout -k 10 570 python3 -u tools/pool_soak.py --seconds 540 > gpurun_out/r03s_long_soak.log 2>&1 &&
NANOPOW_VIRTUAL_DEVICES=8 timeout -k 10 290 python3 -u tools/pool_soak.py --seconds 260 > gpurun_out/r03s_long_soak_8vd.log 2>&1 &&
NANOPOW_LIB=$LIBDIR/libnanopow_ubsan.so UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1 NANOPOW_VIRTUAL_DEVICES=4 timeout -k 10 290 python3 -u tools/pool_soak.py --seconds 260 > gpurun_out/r03s_long_soak_ubsan_4vd.log 2>&1
rc=$?
tail -n 1 gpurun_out/r03s_long_soak*.log
exit $rc
