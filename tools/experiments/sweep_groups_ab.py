#!/usr/bin/env python3
"""Sweep-kernel A/B of lockstep workgroups per CU (NANOPOW_LS_GROUPS=1 vs 2), interleaved, each arm
its own process: a 2^34 exhaustive sweep of the configs[2] fixture root at fffffff8 (exact hit set
checked against tests/golden/sweep_2p36.json), kernel-event and wall rates.
Usage (GPU box): python3 tools/experiments/sweep_groups_ab.py ROUNDS [arm ...]"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
CODE = """
import json, sys, time
sys.path.insert(0, %r)
from nanopow import _lib
fx = json.load(open(%r))
e = _lib.Engine()
root, thr = bytes.fromhex(fx["root"]), int(fx["threshold"], 16)
e.sweep(root, thr, 0, 1 << 30)
e.reset_stats(0)
t = time.perf_counter(); hits = e.sweep(root, thr, 0, 1 << 34); dt = time.perf_counter() - t
st = e.stats(0)
want = [int(h, 16) for h in fx["hits"] if int(h, 16) < 1 << 34]
print(json.dumps({"gnps": round((1 << 34) / dt / 1e9, 4), "kernel_gnps": round(st.nonces / (st.kernel_ms * 1e-3) / 1e9, 4),
                  "exact": hits == want, "hits": len(hits), "clock_mhz": round(st.clock_mhz, 1)}))
""" % (os.path.join(ROOT, "nano-dpow_amd"), os.path.join(ROOT, "tests", "golden", "sweep_2p36.json"))
# arms: "1" / "2" = NANOPOW_LS_GROUPS; any VAR=VALUE = that environment on the default build
ARMS = sys.argv[2:] or ["1", "2"]
for rnd in range(int(sys.argv[1])):
    for arm in ARMS:
        env = dict(os.environ)
        if "=" in arm:
            k, v = arm.split("=", 1)
            env[k] = v
        else:
            env["NANOPOW_LS_GROUPS"] = arm
        p = subprocess.run([sys.executable, "-c", CODE], env=env, capture_output=True, text=True, timeout=120)
        if p.returncode:
            raise SystemExit(p.stderr[-2000:])
        r = json.loads(p.stdout.strip().splitlines()[-1])
        r.update(arm=arm, round=rnd)
        print(json.dumps(r), flush=True)
