#!/usr/bin/env python3
"""Where a short search's kernel time goes (round 5): the regime (bench.py --workload regime) over G devices with
NANOPOW_TRACE_LATENCY=1, whose pool workers print each retired launch's HIP-event span, its clock waves' span on the
GPU's realtime clock (workgroups 0-7: first dispatched) and the gap on that clock since the device's previous launch
ended.  Events minus clock waves = dispatch before the first workgroup runs + the drain after the clock waves end.

    python3 tools/experiments/launch_spans.py G SEARCHES [VAR=VAL ...]   -> one JSON line
"""
import json
import os
import re
import statistics
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
PAT = re.compile(r"nanopow-launch dev (\d+) launch (\d+): events ([\d.]+) clock waves ([\d.]+) us, start ([-\d.]+) us")


def pct(xs, q):
    xs = sorted(xs)
    return xs[min(len(xs) - 1, int(q / 100.0 * len(xs)))] if xs else None


def main():
    g, m = sys.argv[1], int(sys.argv[2])
    env = dict(os.environ, NANOPOW_TRACE_LATENCY="1")
    if int(g) > 1:
        env["NANOPOW_VIRTUAL_DEVICES"] = g
    for kv in sys.argv[3:]:
        k, v = kv.split("=", 1)
        env[k] = v
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--workload", "regime", "--gpus", g, "--steps", str(m),
           "--http-requests", "0"]
    p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    if p.returncode != 0:
        raise SystemExit(p.stderr[-3000:])
    r = json.loads(p.stdout.strip().splitlines()[-1])["node_ttw_8x_regime"]
    per = {}
    for mt in PAT.finditer(p.stderr):
        d = int(mt.group(1))
        per.setdefault(d, []).append((float(mt.group(3)), float(mt.group(4)), float(mt.group(5))))
    out = {"devices": int(g), "searches": m, "env": sys.argv[3:], "kernel_gnps": r["kernel_gnps"],
           "node_over_kernel": r["node_over_kernel"], "per_device_kernel_gnps": r["per_device_kernel_gnps"],
           "late_nonces_losers": r["late_nonces_losers"], "mhz": r["in_kernel_mhz"], "per_device": {}}
    for d, xs in sorted(per.items()):
        xs = xs[len(xs) // 10:]  # past the warm-up searches
        ev = [a for a, _, _ in xs]
        ck = [b for _, b, _ in xs]
        gap = [c for _, _, c in xs if c >= 0]
        out["per_device"][d] = {
            "launches": len(xs), "events_us_mean": round(statistics.mean(ev), 1),
            "clock_waves_us_mean": round(statistics.mean(ck), 1),
            "events_minus_clock_p50": round(pct([a - b for a, b, _ in xs], 50), 1),
            "events_minus_clock_mean": round(statistics.mean([a - b for a, b, _ in xs]), 1),
            "gpu_gap_us_p50": round(pct(gap, 50), 1) if gap else None,
            "gpu_gap_us_mean": round(statistics.mean(gap), 1) if gap else None}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
