#!/usr/bin/env python3
"""Fixed overhead of one first-win search: npow_search at threshold 0 (the first nonce of the
first launch wins) timed at the C ABI, plus receive-difficulty searches for comparison.
Prints one JSON line."""
import json
import os
import statistics
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "nano-dpow_amd"))
from nanopow import _lib  # noqa: E402


def pct(xs, p):
    xs = sorted(xs)
    return xs[min(len(xs) - 1, int(round(p / 100 * (len(xs) - 1))))]


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 300
    eng = _lib.Engine()
    out = {}
    for name, thr in (("fff0", 0xfff0000000000000), ("ffff", 0xffff000000000000), ("receive", 0xfffffe0000000000)):
        ts = []
        for i in range(n + 10):
            root = i.to_bytes(8, "little") * 4
            t = time.perf_counter()
            r = eng.search(root, thr, start=i << 40, device_mask=1)
            dt = time.perf_counter() - t
            assert r.status == _lib.NPOW_OK
            if i >= 10:
                ts.append(dt * 1e3)
        out[name] = {"p10": round(pct(ts, 10), 4), "p50": round(pct(ts, 50), 4), "p90": round(pct(ts, 90), 4),
                     "mean": round(statistics.mean(ts), 4)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
