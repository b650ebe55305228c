"""Interleaved A/B of libnanopow builds in ONE process on the bench workload (first-win searches at
fffffff800000000) and on a no-hit sweep.  LIBS=a.so,b.so ROUNDS=3 N_SEARCH=60."""
import hashlib, json, os, statistics, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', '..', 'nano-dpow_amd'))
from nanopow import _lib
libs = os.environ["LIBS"].split(",")
engines = []
for p in libs:
    _lib._lib = None
    engines.append(_lib.Engine(p))
M64 = (1 << 64) - 1
res = {os.path.basename(p): {"search_gnps": [], "search_kernel_gnps": [], "sweep_kernel_gnps": []} for p in libs}
ns = int(os.environ.get("N_SEARCH", "60"))
for rnd in range(int(os.environ.get("ROUNDS", "3"))):
    for p, e in zip(libs, engines):
        k = os.path.basename(p)
        e.reset_stats(0)
        t = time.time(); nn = 0
        for i in range(ns):
            root = hashlib.blake2b(b"ab" + (rnd * 1000 + i).to_bytes(8, "little"), digest_size=32).digest()
            nn += e.search(root, 0xfffffff800000000, start=i << 40).nonces_done
        dt = time.time() - t
        st = e.stats(0)
        res[k]["search_gnps"].append(round(nn / dt / 1e9, 3))
        res[k]["search_kernel_gnps"].append(round(st.nonces / (st.kernel_ms * 1e-3) / 1e9, 3))
        e.reset_stats(0)
        e.sweep(bytes(range(32)), M64, 1 << 50, 1 << 34)
        st = e.stats(0)
        res[k]["sweep_kernel_gnps"].append(round(st.nonces / (st.kernel_ms * 1e-3) / 1e9, 3))
print(json.dumps({k: {m: statistics.median(v) for m, v in d.items()} for k, d in res.items()}))
print(json.dumps(res))
