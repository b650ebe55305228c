set -e
mkdir -p gpurun_out
NANOPOW_VIRTUAL_DEVICES=4 timeout -k 10 400 python3 bench.py --gpus 4 --steps 40 --warmup 3 --node-searches 300 > gpurun_out/r04i2_inproc_4cu.json 2> gpurun_out/r04i2_inproc_4cu.err &&
NANOPOW_VIRTUAL_DEVICES=8 timeout -k 10 400 python3 bench.py --gpus 8 --steps 40 --warmup 3 --node-searches 300 > gpurun_out/r04i2_inproc_8cu.json 2> gpurun_out/r04i2_inproc_8cu.err
