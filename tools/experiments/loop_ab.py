#!/usr/bin/env python3
"""Round 4: the search loop's per-iteration overhead besides the hash stream (tools/kernel_loop_census.py: 8 VALU,
17 s_nop).  Two of the VALU are v_readlane of the launch's start clock, which the compiler keeps in lanes of a VGPR
(SGPR spill) and reloads at every iteration for the time-budget check, two more read the dead word into SGPRs to
compare it with the entry's generation; the s_nops are the readlane -> SALU hazards.  Arm "loop": the dead word
compared in one v_cmp (a ballot), the budget checked at every fourth iteration (launches end at most ~45 us later
on a 20-ms budget).  Arms, each its own process, interleaved:
  * "loop": the in-tree sources with that patch;
  * "tree": the in-tree library.
Per arm: send-difficulty searches (bench rate, kernel rate, in-kernel clock, SIMD cycles per hash), receive-difficulty
searches one at a time (p50 / p90 wall time at the C ABI) and the mean launch length under a 4-ms budget.

    python3 tools/experiments/loop_ab.py build
    python3 tools/experiments/loop_ab.py run ROUNDS > out.jsonl

Measured (profiles/r04_ab_loop.jsonl, 8 rounds): 4,245.5 against 4,260.7 SIMD cycles per hash, -15.2 in every round;
launches of 4.057 against 4.034 ms under the 4-ms budget.  Kept: the patch is in the tree since the r04j build (so
`build` now needs the sources of git revision f2a7416 or earlier).
"""
import json
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
CSRC = os.path.join(ROOT, "nano-dpow_amd", "csrc")
OUT = os.path.join(ROOT, "build", "abloop")
SEND, RECEIVE = 0xfffffff800000000, 0xfffffe0000000000

PATCH = [
    ("""      const uint64_t now = budget ? __builtin_amdgcn_s_memrealtime() : 0;
""", ""),
    ("""      if (readlane64(dead, 0) == gen) why = 1u;
      const bool late = budget && !c.bounded && (uint32_t)now - (uint32_t)t_start >= budget;""",
     """      if (__ballot(dead == gen) != 0) why = 1u;
      const bool late = budget && !c.bounded && (it0 & 3u) == 0 &&
                        (uint32_t)__builtin_amdgcn_s_memrealtime() - (uint32_t)t_start >= budget;"""),
]


def build():
    d = os.path.join(OUT, "loop")
    shutil.rmtree(d, ignore_errors=True)
    os.makedirs(d)
    shutil.copytree(CSRC, os.path.join(d, "csrc"), ignore=shutil.ignore_patterns("*.o"))
    shutil.rmtree(os.path.join(OUT, "include"), ignore_errors=True)
    shutil.copytree(os.path.join(ROOT, "include"), os.path.join(OUT, "include"))
    p = os.path.join(d, "csrc", "npow_kernel.hip")
    s = open(p).read()
    for old, new in PATCH:
        assert old in s, old
        s = s.replace(old, new)
    open(p, "w").write(s)
    subprocess.run(["make", "-s", "-C", os.path.join(d, "csrc"), "-j4", f"OUT={os.path.join(d, 'libnanopow.so')}"],
                   check=True)
    shutil.rmtree(os.path.join(d, "csrc"))
    print("built loop")


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
e.set_pool_tuning(budget_us=4000)
tok = _lib.CancelToken()
tk = e.submit(bytes(range(32)), (1 << 64) - 1, device_mask=1, cancel=tok)
time.sleep(0.05)
e.reset_stats(0)
time.sleep(0.5)
st = e.stats(0)
tok.set()
tk.wait(10)
out.update(budget4_launch_ms=round(st.kernel_ms / max(1, st.launches), 4))
print(json.dumps(out))
"""


def arm(name, first):
    env = dict(os.environ)
    if name != "tree":
        env["NANOPOW_LIB"] = os.path.join(OUT, name, "libnanopow.so")
    code = f"ROOT = {ROOT!r}\nSEND = {SEND}\nRECEIVE = {RECEIVE}\nFIRST = {first}\n" + ARM
    p = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
    if p.returncode != 0:
        raise SystemExit(f"arm {name} failed: {p.stderr[-2000:]}")
    return json.loads(p.stdout.strip().splitlines()[-1])


def run(rounds):
    names = ["loop", "tree"]
    for rnd in range(rounds):
        order = names if rnd % 2 == 0 else names[::-1]
        for name in order:
            r = arm(name, first=rnd * 1000)
            r.update(arm=name, round=rnd)
            print(json.dumps(r), flush=True)


if __name__ == "__main__":
    if sys.argv[1] == "build":
        build()
    else:
        run(int(sys.argv[2]))
