"""Sweep kernel (npow_task_kernel<kSweep>) throughput at several workgroups-per-CU settings:
exact 2^34-nonce no-hit sweeps.  Usage: python3 tools/experiments/sweep_bpc.py 6,7,8"""
import json, os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "nano-dpow_amd"))
from nanopow import _lib
e = _lib.Engine()
M64 = (1 << 64) - 1
for rep in range(2):
    for bpc in [int(x) for x in sys.argv[1].split(",")]:
        e.set_tuning(0, 0, bpc)
        e.reset_stats(0)
        t = time.perf_counter()
        e.sweep(bytes(range(32)), M64, 1 << 50, 1 << 34)
        dt = time.perf_counter() - t
        st = e.stats(0)
        print(json.dumps({"blocks_per_cu": bpc, "wall_gnps": round((1 << 34) / dt / 1e9, 3),
                          "kernel_gnps": round(st.nonces / (st.kernel_ms * 1e-3) / 1e9, 3)}), flush=True)
