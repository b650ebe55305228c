#!/usr/bin/env python3
"""Nonces per launch against the launch budget, with no win to end a launch early: one search at
threshold 2^64 - 1 (never met in practice) runs ~1.5 s per budget, then is cancelled; the kernel's
event-timed launch durations and nonce counts give the average rate of a launch of each length, and
the marginal rate between consecutive budgets tells whether the late part of a launch is slower.
Prints one JSON line per budget (GPU box)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "nano-dpow_amd"))
from nanopow import _lib  # noqa: E402

M64 = (1 << 64) - 1


def main():
    e = _lib.Engine()
    budgets = [int(x) for x in (sys.argv[1:] or ["2000", "5000", "10000", "20000", "40000", "60000"])]
    prev = None
    for rep in range(2):
        for b in budgets:
            e.set_pool_tuning(budget_us=b)
            e.set_tuning(65536, 0, 0)  # the cap far above any budget here
            e.reset_stats(0)
            tok = _lib.CancelToken()
            t = e.submit(bytes(range(32)), M64, start=rep << 50, device_mask=1, cancel=tok)
            time.sleep(1.5)
            tok.set()
            t.wait(30)
            st = e.stats(0)
            n, ms, L = st.nonces, st.kernel_ms, st.launches
            row = {"budget_us": b, "rep": rep, "launches": L, "avg_launch_ms": round(ms / L, 4),
                   "nonces_per_launch": round(n / L), "kernel_gnps": round(n / (ms * 1e-3) / 1e9, 4),
                   "clock_mhz": round(st.clock_mhz, 1),
                   "cycles_per_hash": round(1024 * 64 * st.clock_mhz * 1e6 / (n / (ms * 1e-3)), 1)}
            if prev and prev[0] < b and prev[3] == rep:
                dn, dt = n / L - prev[1], ms / L - prev[2]
                row["marginal_gnps"] = round(dn / (dt * 1e-3) / 1e9, 4)
            prev = (b, n / L, ms / L, rep)
            print(json.dumps(row), flush=True)
    e.set_tuning(8192, 0, 0)


if __name__ == "__main__":
    main()
