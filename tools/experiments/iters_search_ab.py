"""Same 100 bench searches at two iterations-per-launch settings: winners, nonces hashed and wall
time per search, to see where a longer launch gains.  Usage: python3 tools/experiments/iters_search_ab.py 256 4096"""
import json, os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "nano-dpow_amd"))
import bench
from nanopow import _lib
e = _lib.Engine()
res = {}
for it in [int(x) for x in sys.argv[1:]]:
    e.set_tuning(it, 0, 0)
    for w in range(3):
        e.search(bench.bench_root(999000 + w), bench.SEND, start=bench.bench_start(w))
    e.reset_stats(0)
    rows = []
    for i in range(100):
        t = time.perf_counter()
        r = e.search(bench.bench_root(1_000_000 + i), bench.SEND, start=bench.bench_start(1_000_000 + i))
        rows.append((r.nonce, r.nonces_done, time.perf_counter() - t))
    st = e.stats(0)
    res[it] = rows
    print(json.dumps({"iters": it, "nonces": sum(x[1] for x in rows), "wall": round(sum(x[2] for x in rows), 4),
                      "kernel_ms": round(st.kernel_ms, 2), "dev_nonces": st.nonces, "launches": st.launches}), flush=True)
a, b = [res[int(x)] for x in sys.argv[1:3]]
same = sum(1 for x, y in zip(a, b) if x[0] == y[0])
print(json.dumps({"same_winner": same, "per_search": [(x[1], y[1], round(x[2] * 1e3, 2), round(y[2] * 1e3, 2))
                                                      for x, y in zip(a[:15], b[:15])]}))
