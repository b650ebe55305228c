"""Launch time budget A/B through the engine: an unbounded never-hit job run for a fixed time
(then cancelled) and the bench's first-win searches, at several budgets (0 = iteration count).
Usage: python3 tools/experiments/budget_ab.py 0 5000 [iters]"""
import json, os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "nano-dpow_amd"))
import bench
from nanopow import _lib
e = _lib.Engine()
M64 = (1 << 64) - 1
budgets = [int(x) for x in sys.argv[1].split(",")]
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 0
bpcs = [int(x) for x in sys.argv[3].split(",")] if len(sys.argv) > 3 else [0]
if iters:
    e.set_tuning(iters, 0, 0)
for rep in range(2):
  for bpc in bpcs:
    if bpc:
        e.set_pool_tuning(None, bpc)
    for b in budgets:
        e.set_launch_budget(b)
        e.reset_stats(0)
        tok = _lib.CancelToken()
        t0 = time.perf_counter()
        t = e.submit(bytes(range(32)), M64, start=rep << 60, device_mask=1, cancel=tok)
        time.sleep(2.0)
        tok.set()
        r = t.wait(30)
        dt = time.perf_counter() - t0
        st = e.stats(0)
        nohit = {"wall_gnps": round(r.nonces_done / dt / 1e9, 3),
                 "kernel_gnps": round(st.nonces / (st.kernel_ms * 1e-3) / 1e9, 3),
                 "avg_launch_ms": round(st.kernel_ms / st.launches, 3)}
        e.reset_stats(0)
        t0 = time.perf_counter()
        n = 0
        for i in range(80):
            k = 1_000_000 + rep * 1000 + i
            n += e.search(bench.bench_root(k), bench.SEND, start=bench.bench_start(k), device_mask=1).nonces_done
        dt = time.perf_counter() - t0
        st = e.stats(0)
        print(json.dumps({"blocks_per_cu": bpc, "budget_us": b, "nohit": nohit, "search_wall_gnps": round(n / dt / 1e9, 3),
                          "search_kernel_gnps": round(st.nonces / (st.kernel_ms * 1e-3) / 1e9, 3),
                          "search_avg_launch_ms": round(st.kernel_ms / st.launches, 3)}), flush=True)
