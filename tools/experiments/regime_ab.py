#!/usr/bin/env python3
"""Interleaved A/B of the 8-GPU time regime (bench.py --workload regime), each run its own process (round 5).

Arms are NAME=G[@VAR=VAL...]: G devices (CU partitions of GPU 0 when G > 1: NANOPOW_VIRTUAL_DEVICES=G) and extra
environment for the arm (e.g. w8=8 nw8=8@NANOPOW_WATCHER=0).  Per run: one line with the record's headline figures
(node rate over kernel rate, fixed cost per search, p50 against the expectation, the GPU idle per launch gap and the
host timeline's medians).

    python3 tools/experiments/regime_ab.py ROUNDS SEARCHES w1=1 nw1=1@NANOPOW_WATCHER=0 ... > out.jsonl
"""
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))


def run(name, spec, searches):
    g, *extra = spec.split("@")
    env = dict(os.environ)
    if int(g) > 1:
        env["NANOPOW_VIRTUAL_DEVICES"] = g
    for kv in extra:
        k, v = kv.split("=", 1)
        env[k] = v
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--workload", "regime", "--gpus", g, "--steps",
           str(searches), "--http-requests", "0"]
    p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    if p.returncode != 0:
        raise SystemExit(f"arm {name} failed: {p.stderr[-2000:]}")
    r = json.loads(p.stdout.strip().splitlines()[-1])["node_ttw_8x_regime"]
    d = r["decomposition_us"]

    def p50(k):
        v = d.get(k)
        return v["p50"] if isinstance(v, dict) and "p50" in v else None
    return {"arm": name, "devices": int(g), "node_over_kernel": r["node_over_kernel"], "node_gnps": r["node_gnps"],
            "kernel_gnps": r["kernel_gnps"], "fixed_us": r["fixed_cost_us"]["fixed_us"],
            "reference_gnps": r.get("reference_gnps"), "node_over_reference": r.get("node_over_reference"),
            "fixed_at_reference_us": r.get("fixed_cost_at_reference_us"),
            "p50_minus_expected_at_reference_ms": r.get("p50_minus_expected_at_reference_ms"),
            "p50_ms": r["c_abi_ttw_ms"]["p50"], "p50_minus_expected_ms": r["p50_minus_expected_ms"],
            "idle_us": d["gpu_idle_between_launches"]["mean_per_gap"], "adopt_p50": p50("adopt"),
            "launch_last_p50": p50("launch_last_device"), "win_to_decided_p50": p50("win_seen_to_decided"),
            "decided_to_result_p50": p50("decided_to_result_in_client"),
            "turnaround_p50": p50("client_turnaround_to_next_submit"), "losers_stop_p50": p50("losers_stop_after_decide"),
            "mhz": r["in_kernel_mhz"], "cores": r["worker_core_share"],
            "launches_per_search": r.get("launches_per_search_per_device"),
            "dyn_per_search": r.get("dyn_entries_per_search_per_device")}


def main():
    rounds, searches = int(sys.argv[1]), int(sys.argv[2])
    arms = [a.split("=", 1) for a in sys.argv[3:]]
    for rnd in range(rounds):
        order = arms if rnd % 2 == 0 else arms[::-1]
        for name, spec in order:
            r = run(name, spec, searches)
            r["round"] = rnd
            print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
