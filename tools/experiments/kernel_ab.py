"""Interleaved A/B of kernel throughput: search vs sweep mode, iterations per launch, blocks per CU.
Same work in every arm (threshold 2^64-1: no hits, so no early exit); kernel time from HIP events."""
import json, os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', '..', 'nano-dpow_amd'))
from nanopow import _lib
e = _lib.Engine(os.environ.get("NANOPOW_LIB", _lib.LIB_PATH))
M64 = (1 << 64) - 1
root = bytes(range(32))
N = 1 << 34
res = {}
arms = []
for bpc in [int(x) for x in os.environ.get("BPC", "8").split(",")]:
    for it in [int(x) for x in os.environ.get("ITERS", "64,256").split(",")]:
        for mode in ["search", "sweep"]:
            arms.append((bpc, it, mode))
        arms.append((bpc, it, "benchloop"))
for rnd in range(int(os.environ.get("ROUNDS", "2"))):
    for bpc, it, mode in arms:
        e.set_tuning(it, 64, bpc)
        e.reset_stats(0)
        t = time.time()
        if mode == "benchloop":
            import hashlib
            nn = 0
            t = time.time()
            for i in range(60):
                rt = hashlib.blake2b(b"nanopow-bench" + i.to_bytes(8, "little"), digest_size=32).digest()
                r = e.search(rt, 0xfffffff800000000, start=i << 40)
                nn += r.nonces_done
            dt = time.time() - t
            st = e.stats(0)
            k = f"bpc{bpc}_it{it}_{mode}"
            res.setdefault(k, []).append((round(nn / dt / 1e9, 3), round(st.nonces / (st.kernel_ms * 1e-3) / 1e9, 3), round(st.kernel_ms / st.launches, 3)))
            continue
        if mode == "search":
            r = e.search(root, M64, start=1 << 50, max_nonces_per_device=N)
            assert r.status == _lib.NPOW_EXHAUSTED
        else:
            e.sweep(root, M64, 1 << 50, N)
        dt = time.time() - t
        st = e.stats(0)
        k = f"bpc{bpc}_it{it}_{mode}"
        res.setdefault(k, []).append((round(N / dt / 1e9, 3), round(st.nonces / (st.kernel_ms * 1e-3) / 1e9, 3), round(st.kernel_ms / st.launches, 3)))
print(json.dumps(res))
