#!/usr/bin/env python3
"""Interleaved A/B of libnanopow builds, each arm in its own process (round 5).

Arms are NAME=PATH[@VAR=VAL[@VAR=VAL...]] (PATH = a libnanopow.so; "tree" = the in-tree library; the VAR=VAL pairs go
into that arm's environment, e.g. tree@NANOPOW_WATCHER=0).  Per arm and round: 150
send-difficulty searches one at a time (bench rate, kernel rate, in-kernel clock, SIMD cycles per 64-nonce hash)
and 300 receive-difficulty searches (p50 / p90 wall time at the C ABI).  The order of the arms alternates by round.

    python3 tools/experiments/lib_arms_ab.py ROUNDS r04=build/r04lib/libnanopow.so tree=tree > out.jsonl
"""
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
SEND, RECEIVE = 0xfffffff800000000, 0xfffffe0000000000

ARM = r"""
import hashlib, json, sys, time
sys.path.insert(0, ROOT + "/nano-dpow_amd")
from nanopow import _lib
e = _lib.Engine()
def root(i): return hashlib.blake2b(b"nanopow-bench" + i.to_bytes(8, "little"), digest_size=32).digest()
for i in range(3): e.search(root(10**6 + i), SEND, start=i << 40)
out = {}
e.reset_stats(0)
n = 0
t = time.perf_counter()
for i in range(FIRST, FIRST + 150):
    n += e.search(root(i), SEND, start=i << 40).nonces_done
dt = time.perf_counter() - t
st = e.stats(0)
kg = st.nonces / (st.kernel_ms * 1e-3) / 1e9
out.update(gnps=round(n / dt / 1e9, 4), kernel_gnps=round(kg, 4), clock_mhz=round(st.clock_mhz, 1),
           cycles_per_hash=round(1024 * 64 * st.clock_mhz * 1e6 / (kg * 1e9), 1))
ts = []
for i in range(FIRST, FIRST + 300):
    t = time.perf_counter()
    e.search(root(5 * 10**6 + i), RECEIVE, start=i << 40)
    ts.append((time.perf_counter() - t) * 1e3)
ts.sort()
out.update(receive_p50_ms=round(ts[len(ts) // 2], 4), receive_p90_ms=round(ts[int(len(ts) * 0.9)], 4))
print(json.dumps(out))
"""


def arm(name, spec, first):
    env = dict(os.environ)
    path, *extra = spec.split("@")
    for kv in extra:
        k, v = kv.split("=", 1)
        env[k] = v
    if path != "tree":
        env["NANOPOW_LIB"] = os.path.abspath(path)
    code = f"ROOT = {ROOT!r}\nSEND = {SEND}\nRECEIVE = {RECEIVE}\nFIRST = {first}\n" + ARM
    p = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
    if p.returncode != 0:
        raise SystemExit(f"arm {name} failed: {p.stderr[-2000:]}")
    return json.loads(p.stdout.strip().splitlines()[-1])


def main():
    rounds = int(sys.argv[1])
    arms = [a.split("=", 1) for a in sys.argv[2:]]
    for rnd in range(rounds):
        order = arms if rnd % 2 == 0 else arms[::-1]
        for name, path in order:
            r = arm(name, path, first=rnd * 1000)
            r.update(arm=name, round=rnd)
            print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
