#!/usr/bin/env python3
"""Round 4: where the search loop acts on a stop request (a win, a kill, a dead entry, the budget).
Rounds 2-3 read the workgroup's request word at the top of an iteration but acted on it after that
iteration's hash (one more hash per stop); round 4 acts before the hash.  Arms, each its own process on
the same roots, interleaved over rounds:
  * "after": the search kernel of git revision REV (default HEAD) built beside the tree's other sources;
  * "tree":  the in-tree library.
Per arm: send-difficulty searches (bench rate, kernel rate, in-kernel clock, SIMD cycles per hash),
receive-difficulty searches one at a time (p50 / p90 wall time at the C ABI), and a 4-partition
first-win overshoot sample (NANOPOW_VIRTUAL_DEVICES=4: host-observed stop span, device-side late nonces).

    python3 tools/experiments/stop_ab.py build [REV]
    python3 tools/experiments/stop_ab.py run ROUNDS > out.jsonl
"""
import json
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
CSRC = os.path.join(ROOT, "nano-dpow_amd", "csrc")
OUT = os.path.join(ROOT, "build", "abstop")
SEND, RECEIVE = 0xfffffff800000000, 0xfffffe0000000000


def build(rev="HEAD"):
    d = os.path.join(OUT, "after")
    shutil.rmtree(d, ignore_errors=True)
    os.makedirs(d)
    shutil.copytree(CSRC, os.path.join(d, "csrc"), ignore=shutil.ignore_patterns("*.o"))
    shutil.rmtree(os.path.join(OUT, "include"), ignore_errors=True)
    shutil.copytree(os.path.join(ROOT, "include"), os.path.join(OUT, "include"))
    k = subprocess.run(["git", "show", f"{rev}:nano-dpow_amd/csrc/npow_kernel.hip"], cwd=ROOT, check=True,
                       capture_output=True, text=True).stdout
    assert "(v >> 2) <= it" not in k, "that revision already acts before the hash"
    open(os.path.join(d, "csrc", "npow_kernel.hip"), "w").write(k)
    subprocess.run(["make", "-s", "-C", os.path.join(d, "csrc"), "-j4", f"OUT={os.path.join(d, 'libnanopow.so')}"],
                   check=True)
    shutil.rmtree(os.path.join(d, "csrc"))
    print(f"built after: npow_kernel.hip of {rev}")


ARM = r"""
import hashlib, json, statistics, sys, time
sys.path.insert(0, ROOT + "/nano-dpow_amd")
from nanopow import _lib
e = _lib.Engine()
def root(i): return hashlib.blake2b(b"nanopow-bench" + i.to_bytes(8, "little"), digest_size=32).digest()
for i in range(3): e.search(root(10**6 + i), SEND, start=i << 40)
out = {}
if MODE == "single":
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
        r = e.search(root(5 * 10**6 + i), RECEIVE, start=i << 40)
        ts.append((time.perf_counter() - t) * 1e3)
    ts.sort()
    out.update(receive_p50_ms=round(ts[len(ts) // 2], 4), receive_p90_ms=round(ts[int(len(ts) * 0.9)], 4))
else:
    G = e.n_devices
    spans, late = [], []
    for i in range(FIRST, FIRST + 150):
        t = e.submit(root(7 * 10**6 + i), RECEIVE, start=i << 40, device_mask=0)
        info = t.wait_info(60)
        spans.append(info.stop_after_decide_us)
        late.append(info.late_nonces_losers)
    spans.sort()
    late.sort()
    out.update(devices=G, stop_p50_us=round(spans[len(spans) // 2], 1), stop_p99_us=round(spans[int(len(spans) * 0.99)], 1),
               late_losers_p50=late[len(late) // 2])
print(json.dumps(out))
"""


def arm(name, mode, first):
    env = dict(os.environ)
    if name != "tree":
        env["NANOPOW_LIB"] = os.path.join(OUT, name, "libnanopow.so")
    if mode == "multi":
        env["NANOPOW_VIRTUAL_DEVICES"] = "4"
    code = f"ROOT = {ROOT!r}\nSEND = {SEND}\nRECEIVE = {RECEIVE}\nMODE = {mode!r}\nFIRST = {first}\n" + ARM
    p = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
    if p.returncode != 0:
        raise SystemExit(f"arm {name} {mode} failed: {p.stderr[-2000:]}")
    return json.loads(p.stdout.strip().splitlines()[-1])


def run(rounds):
    names = ["after", "tree"]
    for rnd in range(rounds):
        for mode in ("single", "multi"):
            order = names if rnd % 2 == 0 else names[::-1]
            for name in order:
                r = arm(name, mode, first=rnd * 1000)
                r.update(arm=name, mode=mode, round=rnd)
                print(json.dumps(r), flush=True)


if __name__ == "__main__":
    if sys.argv[1] == "build":
        build(*sys.argv[2:3])
    else:
        run(int(sys.argv[2]))
