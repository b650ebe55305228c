"""A/B helper: parity + sweep throughput of one libnanopow.so variant (NANOPOW_LIB)."""
import os, sys, time, random, json
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', '..', 'nano-dpow_amd'))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', '..', 'oracle'))
import nanopow, oracle
from nanopow import _lib
e = _lib.Engine(os.environ.get("NANOPOW_LIB", _lib.LIB_PATH))
rng = random.Random(7)
root = bytes(rng.getrandbits(8) for _ in range(32))
vals = e.values(root, rng.getrandbits(64), 8192)
ok_vals = True
start = None
res = {"lib": os.path.basename(os.environ.get("NANOPOW_LIB", "default"))}
s0 = rng.getrandbits(64)
vals = e.values(root, s0, 8192)
res["values_ok"] = vals == [oracle.work_value(root, s0 + i) for i in range(8192)]
hits = e.sweep(root, 0xfffff00000000000, 0, 1 << 25)
res["sweep_ok"] = hits == oracle.sweep(root, 0xfffff00000000000, 0, 1 << 25)
for it, poll in [(int(x), int(y)) for x in os.environ.get("ITERS", "64").split(",") for y in os.environ.get("POLL", "64").split(",")]:
    e.set_tuning(it, poll, 0)
    e.sweep(root, 0xfffffff800000000, 0, 1 << 30)  # warm
    e.reset_stats(0)
    t = time.time(); n = 1 << 35; h = e.sweep(root, 0xfffffff800000000, 1 << 40, n); dt = time.time() - t
    st = e.stats(0)
    res[f"iters{it}_poll{poll}"] = {"wall_gnps": round(n / dt / 1e9, 3), "kernel_gnps": round(st.nonces / (st.kernel_ms * 1e-3) / 1e9, 3),
                         "launches": st.launches, "ms_per_launch": round(st.kernel_ms / st.launches, 3), "hits": len(h)}
print(json.dumps(res))
