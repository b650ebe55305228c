#!/bin/bash
# Round-6 closing GPU session, part 3 (the final build): every bench.py workload (BASELINE configs[0]-[4], the MQTT
# path) and the five 60-s pool soaks (one device; 4 partitions; injected invalid work; injected HIP failures; CPU
# workers), each step with its own time limit.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
T=${1:-r06f}
bash tools/workloads_refresh.sh $T &&
bash tools/soaks_r04.sh $T
rc=$?
wc -l gpurun_out/workloads_$T.jsonl
exit $rc
