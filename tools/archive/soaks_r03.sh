#!/bin/bash
# Round-3 pool soaks (tools/pool_soak.py): one device, 4 logical devices, 4 logical devices with
# device 1's wins corrupted, and with device 2's launches failing after its 200th.  Each has its own
# time limit; the chain stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 150 python3 -u tools/pool_soak.py --seconds 60 > gpurun_out/r03_soak.log 2>&1 &&
NANOPOW_VIRTUAL_DEVICES=4 timeout -k 10 150 python3 -u tools/pool_soak.py --seconds 60 > gpurun_out/r03_soak_4vd.log 2>&1 &&
NANOPOW_TEST_HOOKS=1 NANOPOW_VIRTUAL_DEVICES=4 NANOPOW_FAULT_INVALID=1 timeout -k 10 150 python3 -u tools/pool_soak.py --seconds 60 --faults > gpurun_out/r03_soak_fault_invalid.log 2>&1 &&
NANOPOW_TEST_HOOKS=1 NANOPOW_VIRTUAL_DEVICES=4 NANOPOW_FAULT_HIP=2:200 timeout -k 10 150 python3 -u tools/pool_soak.py --seconds 60 --faults > gpurun_out/r03_soak_fault_hip.log 2>&1
rc=$?
tail -n 1 gpurun_out/r03_soak*.log
exit $rc
