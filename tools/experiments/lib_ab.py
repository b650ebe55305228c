"""Interleaved A/B of several libnanopow.so builds in ONE process (guide §5.4 rule 24).
LIBS=a.so,b.so ROUNDS=3 python3 tools/experiments/lib_ab.py -> median kernel Gnonce/s per build (sweep, no hits)."""
import ctypes, json, os, statistics, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', '..', 'nano-dpow_amd'))
from nanopow import _lib
libs = os.environ["LIBS"].split(",")
engines = []
for p in libs:
    _lib._lib = None            # force a fresh CDLL per build
    engines.append(_lib.Engine(p))
M64 = (1 << 64) - 1
N = int(os.environ.get("N", str(1 << 35)))
root = bytes(range(32))
res = {os.path.basename(p): [] for p in libs}
for e in engines:  # warm
    e.sweep(root, M64, 0, 1 << 30)
for rnd in range(int(os.environ.get("ROUNDS", "3"))):
    for p, e in zip(libs, engines):
        e.reset_stats(0)
        e.sweep(root, M64, 1 << 50, N)
        st = e.stats(0)
        res[os.path.basename(p)].append(round(st.nonces / (st.kernel_ms * 1e-3) / 1e9, 3))
print(json.dumps({k: {"median": statistics.median(v), "all": v} for k, v in res.items()}))
