#!/bin/bash
# Round-6 closing GPU session, part 3 (the final build): the host-sanitizer GPU tests on the freshly built sanitizer
# libraries, every bench.py workload (BASELINE configs[0]-[4], the MQTT path) and the five 60-s pool soaks (one
# device; 4 partitions; injected invalid work; injected HIP failures; CPU workers), each step with its own time limit.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-r06f}
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_sanitizers.py -x -v --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest_sanitizers.log 2>&1 &&
bash tools/workloads_refresh.sh $T &&
bash tools/soaks_r04.sh $T
rc=$?
tail -3 gpurun_out/${T}_pytest_sanitizers.log
wc -l gpurun_out/workloads_$T.jsonl
exit $rc
