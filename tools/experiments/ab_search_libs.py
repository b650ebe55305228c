"""Interleaved A/B of two libnanopow builds in ONE process on the bench workload (first-win
searches at fffffff800000000) and a no-hit sweep.  Each build is loaded through its own copy
of the ctypes shim (A_SHIM / B_SHIM: paths of _lib.py files matching each build).
A=path.so B=path.so A_SHIM=... B_SHIM=... ROUNDS=3 N_SEARCH=60 python3 tools/experiments/ab_search_libs.py"""
import hashlib, importlib.util, json, os, statistics, sys, time

M64 = (1 << 64) - 1


def load(shim, so, tag):
    spec = importlib.util.spec_from_file_location(f"shim_{tag}", shim)
    m = importlib.util.module_from_spec(spec)
    sys.modules[spec.name] = m
    spec.loader.exec_module(m)
    return m.Engine(so)


# LIBS=name=path.so:shim.py,name2=... (or the A/B pair via A, A_SHIM, B, B_SHIM)
if "LIBS" in os.environ:
    specs = [x.split("=", 1) for x in os.environ["LIBS"].split(",")]
    engines = {name: load(v.split(":")[1], v.split(":")[0], name) for name, v in specs}
else:
    engines = {k: load(os.environ[k + "_SHIM"], os.environ[k], k) for k in ("A", "B")}
res = {k: {"search_gnps": [], "search_kernel_gnps": [], "sweep_kernel_gnps": [], "nohit_search_kernel_gnps": [],
          "nohit_search_gnps": []} for k in engines}
ns = int(os.environ.get("N_SEARCH", "60"))
for rnd in range(int(os.environ.get("ROUNDS", "3"))):
    for k, e in engines.items():
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
        e.reset_stats(0)
        t = time.time()
        r = e.search(bytes(range(32)), M64, start=1 << 52, max_nonces_per_device=1 << 34)
        dt = time.time() - t
        st = e.stats(0)
        res[k]["nohit_search_kernel_gnps"].append(round(st.nonces / (st.kernel_ms * 1e-3) / 1e9, 3))
        res[k]["nohit_search_gnps"].append(round(r.nonces_done / dt / 1e9, 3))
        print(json.dumps({k: {m: v[-1] for m, v in res[k].items()}}), flush=True)
print(json.dumps({k: {m: statistics.median(v) for m, v in d.items()} for k, d in res.items()}))
