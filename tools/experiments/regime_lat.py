#!/usr/bin/env python3
"""Round-5 probe: the regime workload (bench.py --workload regime: next submit at the previous decision, a reaper
collecting tickets) with NANOPOW_TRACE_LATENCY; medians of the per-search host timeline (nanopow-lat) and the
regime's headline figures -> one JSON line.
    python3 tools/experiments/regime_lat.py G SEARCHES [VAR=VAL ...]"""
import json
import os
import re
import statistics
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))


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
    fields = {}
    for mt in re.finditer(r"nanopow-lat adopt ([-\d.]+) launch ([-\d.]+) win ([-\d.]+) kend ([-\d.]+) finish ([-\d.]+) "
                          r"return ([-\d.]+)", p.stderr):
        for k, v in zip(("adopt", "launch", "win", "kend", "finish", "return"), mt.groups()):
            fields.setdefault(k, []).append(float(v))
    out = {"devices": int(g), "env": sys.argv[3:], "node_over_reference": r.get("node_over_reference"),
           "p50_minus_expected_at_reference_ms": r.get("p50_minus_expected_at_reference_ms"),
           "nonces_per_search_over_E": r.get("nonces_per_search_over_E"), "c_abi_ttw_ms": r["c_abi_ttw_ms"]}
    for k, xs in fields.items():
        xs = xs[len(xs) // 10:]
        out[k + "_p50"] = round(statistics.median(xs), 1)
        out[k + "_mean"] = round(statistics.mean(xs), 1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
