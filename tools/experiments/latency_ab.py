#!/usr/bin/env python3
"""Interleaved A/B of per-search latency: receive-difficulty searches (fffffe00...) and threshold-0
searches (the first hash wins: the fixed per-search cost), each arm its own process on the same
roots, libraries as in setprio_ab.py (build/abprio/<name>/libnanopow.so, "tree", or VAR=VALUE).
  run (GPU box): python3 tools/experiments/latency_ab.py ROUNDS SEARCHES name ..."""
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
OUT = os.path.join(ROOT, "build", "abprio")


def arm(name, n, first):
    env = dict(os.environ)
    if "=" in name:
        k, v = name.split("=", 1)
        env[k] = v
    elif name != "tree":
        env["NANOPOW_LIB"] = os.path.join(OUT, name, "libnanopow.so")
    code = f"""
import hashlib, json, statistics, sys, time
sys.path.insert(0, {os.path.join(ROOT, 'nano-dpow_amd')!r})
from nanopow import _lib
e = _lib.Engine()
def root(i): return hashlib.blake2b(b"nanopow-lat" + i.to_bytes(8, "little"), digest_size=32).digest()
for i in range(20): e.search(root(10**7 + i), 0xfffffe0000000000, start=i << 40)
out = {{}}
for thr, tag in ((0xfffffe0000000000, "receive"), (0, "thr0")):
    ts = []
    for i in range({first}, {first} + {n}):
        t = time.perf_counter()
        r = e.search(root(i), thr, start=i << 40)
        ts.append(time.perf_counter() - t)
        assert r.status == 0
    ts.sort()
    out[tag + "_p50_ms"] = round(ts[len(ts) // 2] * 1e3, 4)
    out[tag + "_mean_ms"] = round(statistics.mean(ts) * 1e3, 4)
print(json.dumps(out))
"""
    p = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
    if p.returncode != 0:
        raise SystemExit(f"arm {name} failed: {p.stderr[-2000:]}")
    return json.loads(p.stdout.strip().splitlines()[-1])


def main(rounds, n, names):
    for rnd in range(rounds):
        order = names[rnd % len(names):] + names[:rnd % len(names)]
        for name in order:
            r = arm(name, n, first=rnd * n)
            r.update(arm=name, round=rnd)
            print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main(int(sys.argv[1]), int(sys.argv[2]), sys.argv[3:])
