#!/usr/bin/env python3
"""Interleaved A/B of compile-time variants of the search kernel (round 3: static s_setprio).

  build (here):  python3 tools/experiments/setprio_ab.py build name='-DFLAG=V ...' ...
                 -> build/abprio/<name>/libnanopow.so: the in-tree sources compiled with those flags
                    (nano-dpow_amd/csrc/Makefile EXTRA=...)
  run (GPU box): python3 tools/experiments/setprio_ab.py run ROUNDS SEARCHES name ...
                 -> one JSON line per (round, arm): first-win searches at fffffff800000000 on bench.py's
                    roots, each arm in its own process, the arms' order rotated every round, every
                    (root, nonce) re-checked with hashlib; cycles per hash = 1,024 SIMDs x 64 x the
                    in-kernel clock / the kernel rate.
NPOW_LS2_PRIO (npow_kernel.hip): 1 = s_setprio 1 for the second-dispatched workgroup of each CU,
2 = for waves 8..15 of every workgroup, 3 = waves 0..7 (control for 2).
"""
import json
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
CSRC = os.path.join(ROOT, "nano-dpow_amd", "csrc")
OUT = os.path.join(ROOT, "build", "abprio")
SEND = 0xfffffff800000000


def build(specs):
    for spec in specs:
        name, flags = spec.split("=", 1)
        d = os.path.join(OUT, name)
        shutil.rmtree(d, ignore_errors=True)
        os.makedirs(d)
        shutil.copytree(CSRC, os.path.join(d, "csrc"), ignore=shutil.ignore_patterns("*.o"))
        shutil.copytree(os.path.join(ROOT, "include"), os.path.join(OUT, "include"), dirs_exist_ok=True)
        subprocess.run(["make", "-s", "-C", os.path.join(d, "csrc"), "-j4", f"EXTRA={flags}",
                        f"OUT={os.path.join(d, 'libnanopow.so')}"], check=True)
        shutil.rmtree(os.path.join(d, "csrc"))
        print(f"built {name}: {flags!r}")


def arm(name, searches, first):
    env = dict(os.environ)
    if name != "tree":
        env["NANOPOW_LIB"] = os.path.join(OUT, name, "libnanopow.so")
    code = f"""
import hashlib, json, sys, time
sys.path.insert(0, {os.path.join(ROOT, 'nano-dpow_amd')!r})
from nanopow import _lib
e = _lib.Engine()
def root(i): return hashlib.blake2b(b"nanopow-bench" + i.to_bytes(8, "little"), digest_size=32).digest()
for i in range(3): e.search(root(10**6 + i), {SEND}, start=i << 40)
e.reset_stats(0)
n = 0; bad = 0
t = time.perf_counter()
for i in range({first}, {first} + {searches}):
    r = e.search(root(i), {SEND}, start=i << 40)
    n += r.nonces_done
    v = int.from_bytes(hashlib.blake2b(r.nonce.to_bytes(8, "little") + root(i), digest_size=8).digest(), "little")
    bad += (v != r.value or v < {SEND})
dt = time.perf_counter() - t
st = e.stats(0)
kg = st.nonces / (st.kernel_ms * 1e-3) / 1e9
print(json.dumps({{"gnps": round(n / dt / 1e9, 4), "kernel_gnps": round(kg, 4), "clock_mhz": round(st.clock_mhz, 1),
                  "cycles_per_hash": round(1024 * 64 * st.clock_mhz * 1e6 / (kg * 1e9), 1),
                  "bad": bad, "searches": {searches}}}))
"""
    p = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
    if p.returncode != 0:
        raise SystemExit(f"arm {name} failed: {p.stderr[-2000:]}")
    return json.loads(p.stdout.strip().splitlines()[-1])


def run(rounds, searches, names):
    for rnd in range(rounds):
        order = names[rnd % len(names):] + names[:rnd % len(names)]
        for name in order:
            r = arm(name, searches, first=rnd * searches)  # the same roots for every arm of a round
            r.update(arm=name, round=rnd)
            print(json.dumps(r), flush=True)


if __name__ == "__main__":
    if sys.argv[1] == "build":
        build(sys.argv[2:])
    else:
        run(int(sys.argv[2]), int(sys.argv[3]), sys.argv[4:])
