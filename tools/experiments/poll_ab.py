"""Sweep (no hits) kernel rate at several host-abort poll intervals, one process, plus cancel latency."""
import json, os, sys, threading, time
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', '..', 'nano-dpow_amd'))
from nanopow import _lib
e = _lib.Engine(os.environ.get("NANOPOW_LIB", _lib.LIB_PATH))
M64 = (1 << 64) - 1
root = bytes(range(32))
e.sweep(root, M64, 0, 1 << 32)  # warm the clock
res = {}
for rnd in range(2):
    for poll in [64, 1024, 4096, 1 << 20]:
        e.set_tuning(0, poll, 0)
        e.reset_stats(0)
        e.sweep(root, M64, 1 << 50, 1 << 34)
        st = e.stats(0)
        res.setdefault(poll, []).append(round(st.nonces / (st.kernel_ms * 1e-3) / 1e9, 3))
lat = {}
for poll in [64, 4096]:
    e.set_tuning(0, poll, 0)
    ts = []
    for k in range(5):
        tok = _lib.CancelToken()
        box = {}
        th = threading.Thread(target=lambda: box.setdefault("r", e.search(root, M64, cancel=tok)))
        th.start(); time.sleep(0.05)
        t0 = time.perf_counter(); tok.set(); th.join()
        ts.append(round((time.perf_counter() - t0) * 1e3, 3))
    lat[poll] = ts
print(json.dumps({"kernel_gnps_by_poll": res, "cancel_latency_ms": lat}))
