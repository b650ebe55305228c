# Pool soaks on the final build: one device, 4 logical devices, 4 logical devices with device 1's wins
# corrupted (dropped after 3); 60 s each.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 150 python3 -u tools/pool_soak.py --seconds 60 > gpurun_out/fsoak.log 2>&1 || exit 1
NANOPOW_VIRTUAL_DEVICES=4 timeout -k 10 150 python3 -u tools/pool_soak.py --seconds 60 > gpurun_out/fsoak_4vd.log 2>&1 || exit 1
NANOPOW_VIRTUAL_DEVICES=4 NANOPOW_FAULT_INVALID=1 timeout -k 10 150 python3 -u tools/pool_soak.py --seconds 60 --faults > gpurun_out/fsoak_fault.log 2>&1 || exit 1
tail -n 1 gpurun_out/fsoak.log gpurun_out/fsoak_4vd.log gpurun_out/fsoak_fault.log
