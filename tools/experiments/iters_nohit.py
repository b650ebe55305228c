"""No-hit bounded searches (threshold 2^64-1, exact 2^34 nonces) through the engine at several
iterations per launch: kernel and wall Gnonce/s, to separate steady-state rate from per-search
effects.  Usage: python3 tools/experiments/iters_nohit.py 256 1024 4096"""
import json, os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "nano-dpow_amd"))
from nanopow import _lib
e = _lib.Engine()
M64 = (1 << 64) - 1
for rep in range(2):
    for it in [int(x) for x in sys.argv[1:]]:
        e.set_tuning(it, 0, 0)
        e.reset_stats(0)
        t = time.perf_counter()
        r = e.search(bytes(range(32)), M64, start=1 << 52, max_nonces_per_device=1 << 34)
        dt = time.perf_counter() - t
        st = e.stats(0)
        print(json.dumps({"iters": it, "wall_gnps": round(r.nonces_done / dt / 1e9, 3),
                          "kernel_gnps": round(st.nonces / (st.kernel_ms * 1e-3) / 1e9, 3),
                          "launches": st.launches}), flush=True)
