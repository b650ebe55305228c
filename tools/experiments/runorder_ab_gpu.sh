#!/bin/bash
# Round 3: op order inside the stream's runs (gen_hash_asm.py --run-order): same instructions, same
# schedule shape; does the order change the power-limited clock?
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python3 tools/experiments/setprio_ab.py run 4 150 tree ro_rev ro_s1 ro_s2 ro_s3 > gpurun_out/r03_ab_runorder.jsonl 2> gpurun_out/r03_ab_runorder.err
rc=$?
cat gpurun_out/r03_ab_runorder.jsonl; tail -3 gpurun_out/r03_ab_runorder.err
exit $rc
