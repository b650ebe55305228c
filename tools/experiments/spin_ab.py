#!/usr/bin/env python3
"""Round 4: how often a spinning pool worker asks the HIP runtime whether its launch has ended.  While it
spins (a launch's first 0.4 ms, and 2 ms after one of its jobs stopped) a worker runs a step -- at least
one hipEventQuery -- after every single `pause`; over 8 CU partitions of one GPU, 8 workers do that against
one HIP runtime and the host-observed stop of a split search's losers took ~0.34 ms (p50) against ~0.09 ms
over 4.  Arms (each its own process, interleaved): the in-tree library ("tree") and builds whose spin waits
GAP microseconds between steps (busy, with `pause`): "gap2", "gap5", "gap10".  Per arm: the overshoot sample
over 8 and 4 partitions (host-observed stop span, result time) and receive-difficulty searches on the whole
GPU (p50 / p90 wall time to the result).

    python3 tools/experiments/spin_ab.py build gap2 gap5 gap10
    python3 tools/experiments/spin_ab.py run ROUNDS tree gap2 gap5 gap10 > out.jsonl
"""
import json
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
CSRC = os.path.join(ROOT, "nano-dpow_amd", "csrc")
OUT = os.path.join(ROOT, "build", "abspin")

SPIN_OLD = """    if (sl.state == SlotState::kDraining && sl.stop_us > 0 && !sl.fin_seen && t - sl.stop_us < kStopSpinUs) {
      cpu_relax();
      return;
    }"""
FRESH_OLD = """  if (since < kFreshSpinUs) {
    cpu_relax();
    return;
  }"""


def gap(us):
    return f"""{{
      const double g0_ = now_us();
      while (now_us() - g0_ < {us}.0) cpu_relax();
      return;
    }}"""


def build(names):
    for name in names:
        us = int(name[3:])
        d = os.path.join(OUT, name)
        shutil.rmtree(d, ignore_errors=True)
        os.makedirs(d)
        shutil.copytree(CSRC, os.path.join(d, "csrc"), ignore=shutil.ignore_patterns("*.o"))
        shutil.rmtree(os.path.join(OUT, "include"), ignore_errors=True)
        shutil.copytree(os.path.join(ROOT, "include"), os.path.join(OUT, "include"))
        p = os.path.join(d, "csrc", "npow_pool.cpp")
        s = open(p).read()
        assert SPIN_OLD in s and FRESH_OLD in s
        s = s.replace(SPIN_OLD, SPIN_OLD.replace("{\n      cpu_relax();\n      return;\n    }", gap(us)))
        s = s.replace(FRESH_OLD, "  if (since < kFreshSpinUs) " + gap(us).replace("\n      ", "\n    ").replace("\n    }", "\n  }"))
        open(p, "w").write(s)
        subprocess.run(["make", "-s", "-C", os.path.join(d, "csrc"), "-j4", f"OUT={os.path.join(d, 'libnanopow.so')}"],
                       check=True)
        shutil.rmtree(os.path.join(d, "csrc"))
        print(f"built {name}: {us}-us gaps between spinning steps")


RECV = r"""
import hashlib, json, sys, time
sys.path.insert(0, ROOT + "/nano-dpow_amd")
from nanopow import _lib
e = _lib.Engine()
def root(i): return hashlib.blake2b(b"nanopow-bench" + i.to_bytes(8, "little"), digest_size=32).digest()
for i in range(3): e.search(root(10**6 + i), 0xfffffe0000000000, start=i << 40)
ts = []
for i in range(300):
    t0 = time.perf_counter()
    t = e.submit(root(5 * 10**6 + i), 0xfffffe0000000000, start=i << 40, device_mask=1)
    t.wait_result()
    ts.append((time.perf_counter() - t0) * 1e3)
    t.wait()
ts.sort()
print(json.dumps({"receive_p50_ms": round(ts[150], 4), "receive_p90_ms": round(ts[270], 4)}))
"""


def arm(name, mode):
    env = dict(os.environ)
    if name != "tree":
        env["NANOPOW_LIB"] = os.path.join(OUT, name, "libnanopow.so")
    if mode == "recv":
        cmd = [sys.executable, "-c", f"ROOT = {ROOT!r}\n" + RECV]
    else:
        env["NANOPOW_VIRTUAL_DEVICES"] = mode
        cmd = [sys.executable, os.path.join(ROOT, "tests", "overshoot_worker.py"), "100", "receive"]
    p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    if p.returncode != 0:
        raise SystemExit(f"arm {name} {mode} failed: {p.stderr[-2000:]}")
    out = json.loads(p.stdout.strip().splitlines()[-1])
    keep = ("stop_after_decide_us", "finish_ms_p50", "result_ms_p50", "late_nonces_losers", "receive_p50_ms",
            "receive_p90_ms")
    return {k: out[k] for k in keep if k in out}


def run(rounds, names):
    for rnd in range(rounds):
        for mode in ("8", "4", "recv"):
            order = names[rnd % len(names):] + names[:rnd % len(names)]
            for name in order:
                r = arm(name, mode)
                r.update(arm=name, mode=mode, round=rnd)
                print(json.dumps(r), flush=True)


if __name__ == "__main__":
    if sys.argv[1] == "build":
        build(sys.argv[2:])
    else:
        run(int(sys.argv[2]), sys.argv[3:])
