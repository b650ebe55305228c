"""Child process of tests/test_gpu_multidevice.py: BASELINE configs[2] at full size split over G
devices.  Run with NANOPOW_VIRTUAL_DEVICES=G (G logical devices over the one physical GPU, each with
its own stream, buffers and worker): npow_sweep of [0, 2^36) for the fixture root at fffffff8 over
every device (contiguous count/G sub-ranges, npow_engine.cpp npow_sweep), so fixture hits straddle
the sub-range boundaries the engine cuts.  The hit set must equal tests/golden/sweep_2p36.json (C
oracle, every hit re-hashed by hashlib; the whole range pinned by a hashlib-only scan) and the
devices' nonce counters must add up to exactly 2^36, each device holding its count/G share.
Prints one JSON line; exits non-zero on any mismatch."""
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(ROOT, "nano-dpow_amd"))

from nanopow import _lib  # noqa: E402


def main():
    with open(os.path.join(HERE, "golden", "sweep_2p36.json")) as f:
        g = json.load(f)
    eng = _lib.Engine()
    G = eng.n_devices
    want = os.environ.get("EXPECT_DEVICES") or os.environ.get("NANOPOW_VIRTUAL_DEVICES")
    assert want is None or G == int(want), G
    root, thr, count = bytes.fromhex(g["root"]), int(g["threshold"], 16), g["count"]
    for d in range(G):
        eng.reset_stats(d)
    t = time.perf_counter()
    hits = eng.sweep(root, thr, 0, count, device_mask=0, cap=1 << 12)
    dt = time.perf_counter() - t
    want = [int(h, 16) for h in g["hits"]]
    assert hits == want, (len(hits), len(want), sorted(set(hits) ^ set(want))[:8])
    per = [eng.stats(d).nonces for d in range(G)]
    share = [count // G + (1 if d < count % G else 0) for d in range(G)]
    assert per == share, (per, share)
    assert sum(per) == count
    # which fixture hits lie in which device's sub-range (the boundaries the split cuts)
    bounds = [sum(share[:d]) for d in range(G + 1)]
    per_dev_hits = [sum(1 for h in want if bounds[d] <= h < bounds[d + 1]) for d in range(G)]
    print(json.dumps({"ok": True, "devices": G, "hits": len(hits), "seconds": round(dt, 3),
                      "partitions": [[eng.stats(d).hip_device, eng.stats(d).cu_first, eng.stats(d).cus]
                                     for d in range(G)],
                      "gnps": round(count / dt / 1e9, 3), "nonces_per_device": per,
                      "hits_per_device": per_dev_hits,
                      "affinity": [sum(eng.stats(d).affinity_checks for d in range(G)),
                                   sum(eng.stats(d).affinity_failures for d in range(G))]}), flush=True)


if __name__ == "__main__":
    main()
