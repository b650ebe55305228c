#!/usr/bin/env python3
"""Energy per hash of search-kernel shapes (round 4): the GPU runs the shipped kernel at
its power cap (in-kernel clock 2,150-2,360 MHz by box against 2,400), so the question is hashes per joule,
not cycles per hash alone.  Arms are builds of the current sources with a different number of 512-lane
workgroups per CU (kLsGroups: 4 ships = 8 waves per SIMD; 3 = 6; 2 = 4): fewer waves per SIMD issue
fewer co-issued pairs per cycle (less switching per cycle), so the clock may rise under the same cap.
Each arm runs in its own process on the same roots, interleaved over rounds; per arm: the bench rate,
the kernel rate, the in-kernel clock, SIMD cycles per 64-nonce wave-hash, the card's hwmon power
(sampled every 25 ms) and joules per Gnonce = mean W / kernel Gnonce/s.

    python3 tools/experiments/energy_ab.py build g4 g3 g2
    python3 tools/experiments/energy_ab.py run ROUNDS SEARCHES g4 g3 g2 > out.jsonl
"""
import glob
import json
import os
import re
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
CSRC = os.path.join(ROOT, "nano-dpow_amd", "csrc")
OUT = os.path.join(ROOT, "build", "abenergy")
SEND = 0xfffffff800000000


def build(names):
    for name in names:
        groups = int(name[1:])  # gN: N workgroups per CU
        d = os.path.join(OUT, name)
        shutil.rmtree(d, ignore_errors=True)
        os.makedirs(d)
        shutil.copytree(CSRC, os.path.join(d, "csrc"), ignore=shutil.ignore_patterns("*.o"))
        # the sources include "../../include/nanopow.h": from OUT/<name>/csrc that is OUT/include
        shutil.rmtree(os.path.join(OUT, "include"), ignore_errors=True)
        shutil.copytree(os.path.join(ROOT, "include"), os.path.join(OUT, "include"))
        h = os.path.join(d, "csrc", "npow_internal.h")
        txt = open(h).read()
        txt2 = re.sub(r"constexpr int kLsGroups = \d+;", f"constexpr int kLsGroups = {groups};", txt)
        assert txt2 != txt or groups == 4
        open(h, "w").write(txt2)
        subprocess.run(["make", "-s", "-C", os.path.join(d, "csrc"), "-j4",
                        f"OUT={os.path.join(d, 'libnanopow.so')}"], check=True)
        shutil.rmtree(os.path.join(d, "csrc"))
        print(f"built {name}: {groups} workgroups per CU")


def arm(name, searches, first):
    env = dict(os.environ, NANOPOW_LIB=os.path.join(OUT, name, "libnanopow.so"))
    code = f"""
import hashlib, json, sys, time
sys.path.insert(0, {ROOT!r})
sys.path.insert(0, {os.path.join(ROOT, 'nano-dpow_amd')!r})
import bench
from nanopow import _lib
e = _lib.Engine()
def root(i): return hashlib.blake2b(b"nanopow-bench" + i.to_bytes(8, "little"), digest_size=32).digest()
for i in range(3): e.search(root(10**6 + i), {SEND}, start=i << 40)
e.reset_stats(0)
n = 0; bad = 0
with bench.SclkSampler(0, period=0.025, span="over the arm's searches") as smp:
    t = time.perf_counter()
    for i in range({first}, {first} + {searches}):
        r = e.search(root(i), {SEND}, start=i << 40)
        n += r.nonces_done
        v = int.from_bytes(hashlib.blake2b(r.nonce.to_bytes(8, "little") + root(i), digest_size=8).digest(), "little")
        bad += (v != r.value or v < {SEND})
    dt = time.perf_counter() - t
st = e.stats(0)
kg = st.nonces / (st.kernel_ms * 1e-3) / 1e9
pw = smp.power_summary() or {{}}
print(json.dumps({{"gnps": round(n / dt / 1e9, 4), "kernel_gnps": round(kg, 4), "clock_mhz": round(st.clock_mhz, 1),
                  "cycles_per_hash": round(1024 * 64 * st.clock_mhz * 1e6 / (kg * 1e9), 1),
                  "grid": st.grid, "power_w": pw.get("mean"), "power_max_w": pw.get("max"), "cap_w": pw.get("cap"),
                  "power_samples": pw.get("samples"),
                  "joule_per_gnonce": round(pw["mean"] / kg, 3) if pw.get("mean") else None,
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
