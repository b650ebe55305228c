set -o pipefail
export TMPDIR=/tmp
env | grep -i visible > gpurun_out/r03f_visible_env.txt
timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 40 --warmup 3 --node-searches 100 > gpurun_out/r03f_torchrun2_shared_gpu.json 2> gpurun_out/r03f_torchrun2.err &&
timeout -k 10 400 python3 bench.py --workload receive --steps 300 > gpurun_out/r03f_receive.json 2> gpurun_out/r03f_receive.err
rc=$?; cat gpurun_out/r03f_visible_env.txt; head -c 300 gpurun_out/r03f_torchrun2_shared_gpu.json; tail -3 gpurun_out/r03f_torchrun2.err; exit $rc
