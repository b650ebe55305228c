#!/usr/bin/env python3
"""Round-5 analysis of a diagnostic-library run (NANOPOW_TRACE_LATENCY, -DNPOW_DIAG_TIMES): for consecutive searches
on each device, the GPU time from one search's win to the next search's last workgroup start, the host time from the
win seen to the next search's launch / dynamic entry, and their difference (publish -> last join).
    python3 tools/experiments/join_gaps.py STDERR_FILE [REGIME_JSON]"""
import json
import re
import statistics
import sys


def pct(xs, q):
    xs = sorted(xs)
    return xs[int(q / 100 * (len(xs) - 1))] if xs else None


def main():
    recs = {}
    for line in open(sys.argv[1]):
        m = re.search(r"nanopow-join dev (\d+) ticket (\d+): gpu_join (\d+) gpu_win (\d+) host_launch ([-\d.]+) "
                      r"host_win_seen ([-\d.]+)", line)
        if m:
            recs.setdefault(int(m.group(1)), {})[int(m.group(2))] = (
                int(m.group(3)), int(m.group(4)), float(m.group(5)), float(m.group(6)))
    gaps, host, pick = [], [], []
    for r in recs.values():
        for a in sorted(r):
            if a + 1 not in r:
                continue
            _, wa, _, sa = r[a]
            jb, _, lb, _ = r[a + 1]
            if wa == 0 or jb == 0:
                continue
            g = (jb - wa) / 100.0
            if 0 < g < 5000:
                gaps.append(g)
                host.append(lb - sa)
                pick.append(g - (lb - sa))
    out = {"file": sys.argv[1], "pairs": len(gaps), "win_to_next_last_join_us": {"p50": pct(gaps, 50), "mean": round(
        statistics.mean(gaps), 1)}, "host_win_seen_to_publish_us_p50": pct(host, 50),
        "publish_to_last_join_us": {"p50": round(pct(pick, 50), 1), "p90": round(pct(pick, 90), 1)}}
    if len(sys.argv) > 2:
        reg = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])["node_ttw_8x_regime"]
        out["node_over_reference"] = reg.get("node_over_reference")
    print(json.dumps(out))


if __name__ == "__main__":
    main()
