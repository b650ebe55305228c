# Two-rank torchrun rehearsal on the final build, then the fixed per-search overhead (latency_probe)
# and per-job host timelines (NANOPOW_TRACE_LATENCY) for the final build and build/abls/prev.
set -o pipefail
mkdir -p gpurun_out
HIP_VISIBLE_DEVICES=0 timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 5 > gpurun_out/torchrun2_final.txt 2>&1 || exit 1
tail -n 1 gpurun_out/torchrun2_final.txt
for arm in tree prev; do
  L=""; [ $arm = prev ] && L=$PWD/build/abls/prev/libnanopow.so
  NANOPOW_LIB=${L:-$PWD/nano-dpow_amd/nanopow/libnanopow.so} timeout -k 10 120 python3 tools/latency_probe.py 300 > gpurun_out/lat_$arm.json || exit 1
  NANOPOW_LIB=${L:-$PWD/nano-dpow_amd/nanopow/libnanopow.so} NANOPOW_TRACE_LATENCY=1 timeout -k 10 60 python3 -c "
import sys; sys.path.insert(0, 'nano-dpow_amd')
from nanopow import _lib
e = _lib.Engine()
for i in range(40): e.search(i.to_bytes(8, 'little') * 4, 0xfffffe0000000000, start=i << 40, device_mask=1)
" 2> gpurun_out/trace_$arm.txt || exit 1
done
cat gpurun_out/lat_tree.json gpurun_out/lat_prev.json
