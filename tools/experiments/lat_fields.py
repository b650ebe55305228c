#!/usr/bin/env python3
"""Round-5 probe: serial searches on the devices of this process (NANOPOW_VIRTUAL_DEVICES as set) at a threshold,
NANOPOW_TRACE_LATENCY on; medians of the per-search host timeline (nanopow-lat: adopt, launch issued / dynamic entry
published, win seen, kernel end, finish, return; us since submit) -> one JSON line.
    python3 tools/experiments/lat_fields.py SEARCHES THRESHOLD_HEX [VAR=VAL ...]"""
import json
import os
import re
import statistics
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
CHILD = r"""
import random, sys
sys.path.insert(0, ROOT + "/nano-dpow_amd")
import nanopow
eng = nanopow.engine()
mask = (1 << eng.n_devices) - 1
rng = random.Random(3)
for i in range(N):
    r = bytes(rng.getrandbits(8) for _ in range(32))
    res = eng.submit(r, THR, start=i << 40, device_mask=mask).wait(30)
    assert res.status == 0
"""


def main():
    n, thr = int(sys.argv[1]), int(sys.argv[2], 16)
    env = dict(os.environ, NANOPOW_TRACE_LATENCY="1")
    for kv in sys.argv[3:]:
        k, v = kv.split("=", 1)
        env[k] = v
    code = f"ROOT = {ROOT!r}\nN = {n}\nTHR = {thr}\n" + CHILD
    p = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
    if p.returncode != 0:
        raise SystemExit(p.stderr[-3000:])
    if os.environ.get("LAT_STDERR"):  # keep the child's trace for other analyses
        with open(os.environ["LAT_STDERR"], "w") as f:
            f.write(p.stderr)
    fields = {}
    for m in re.finditer(r"nanopow-lat adopt ([-\d.]+) launch ([-\d.]+) win ([-\d.]+) kend ([-\d.]+) finish ([-\d.]+) "
                         r"return ([-\d.]+)", p.stderr):
        for k, v in zip(("adopt", "launch", "win", "kend", "finish", "return"), m.groups()):
            fields.setdefault(k, []).append(float(v))
    out = {"env": sys.argv[3:], "searches": n, "threshold": sys.argv[2]}
    for k, xs in fields.items():
        xs = xs[len(xs) // 10:]
        out[k + "_p50"] = round(statistics.median(xs), 1)
        out[k + "_mean"] = round(statistics.mean(xs), 1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
