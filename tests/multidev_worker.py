"""Child process of tests/test_gpu_multidevice.py: the multi-device first-win path, on one physical GPU
exposed as NANOPOW_VIRTUAL_DEVICES logical devices (each a CU partition with its own stream, buffers
and pool worker) or on every physical GPU of the box (EXPECT_DEVICES).  Argument "burst": only a burst
of 64 roots split over every device.  Prints one JSON line; exits non-zero on any mismatch."""
import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(ROOT, "nano-dpow_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import oracle  # noqa: E402  (the checker)
from nanopow import _lib  # noqa: E402

M64 = (1 << 64) - 1
RECEIVE, LOW = 0xfffffe0000000000, 0xfffff00000000000


def partitions(eng, G):
    """[hip_device, cu_first, cus] per logical device; logical devices sharing a HIP device must hold
    disjoint CU ranges that cover it (NANOPOW_VIRTUAL_DEVICES: CU-masked streams, npow_engine.cpp)."""
    parts = [[eng.stats(d).hip_device, eng.stats(d).cu_first, eng.stats(d).cus] for d in range(G)]
    by_dev = {}
    for hip, first, cus in parts:
        by_dev.setdefault(hip, []).append((first, cus))
    for hip, lst in by_dev.items():
        if len(lst) > 1 and all(f >= 0 for f, _ in lst):
            lst.sort()
            assert all(a[0] + a[1] == b[0] for a, b in zip(lst, lst[1:])), lst  # disjoint, contiguous
            assert len({c for _, c in lst}) == 1, lst                            # equal shares
    return parts


def burst(eng, G, n=64):
    """n roots in flight at once, each split over every device: all valid (hashlib)."""
    rng = random.Random(17)
    roots = [bytes(rng.getrandbits(8) for _ in range(32)) for _ in range(n)]
    ts = [eng.submit(rt, RECEIVE, start=rng.getrandbits(64), device_mask=0) for rt in roots]
    for rt, t in zip(roots, ts):
        r = t.wait(60)
        assert r.status == _lib.NPOW_OK and oracle.work_value_hashlib(rt, r.nonce) == r.value >= RECEIVE


def main():
    eng = _lib.Engine()
    G = eng.n_devices
    want = os.environ.get("EXPECT_DEVICES") or os.environ.get("NANOPOW_VIRTUAL_DEVICES")
    assert want is None or G == int(want), G
    out = {"devices": G, "partitions": partitions(eng, G)}
    if len(sys.argv) > 1 and sys.argv[1] == "burst":
        for d in range(G):
            eng.reset_stats(d)
        burst(eng, G)
        out["launches_per_device"] = [eng.stats(d).launches for d in range(G)]
        assert all(x > 0 for x in out["launches_per_device"]), out
        out["affinity"] = [sum(eng.stats(d).affinity_checks for d in range(G)),
                           sum(eng.stats(d).affinity_failures for d in range(G))]
        out["ok"] = True
        print(json.dumps(out), flush=True)
        return
    spacing = (1 << 64) // G
    for d in range(G):
        eng.reset_stats(d)
    # 1. searches over every device: valid winners, every device launched
    rng = random.Random(3)
    for _ in range(16):
        root = bytes(rng.getrandbits(8) for _ in range(32))
        r = eng.search(root, RECEIVE, start=rng.getrandbits(64), device_mask=0)
        assert r.status == _lib.NPOW_OK and oracle.work_value_hashlib(root, r.nonce) == r.value >= RECEIVE
    launches = [eng.stats(d).launches for d in range(G)]
    assert all(x > 0 for x in launches), launches
    out["launches_per_device"] = launches
    # 2. exhaustion: each device hashes exactly its own bounded stride
    r = eng.search(bytes(32), M64, start=12345, device_mask=0, max_nonces_per_device=100_003)
    assert r.status == _lib.NPOW_EXHAUSTED and r.nonces_done == G * 100_003, r
    # 3. the winner comes from the stride that holds the only hit: device 2's first nonce has a
    #    high value; every device hashes exactly one nonce at threshold = that value
    root = bytes(range(50, 82))
    base = 777
    x = None
    for i in range(1 << 20):
        n = (base + 2 * spacing + i) & M64
        if oracle.work_value(root, n) >= 0xffff000000000000:
            x = n
            break
    assert x is not None
    vx = oracle.work_value(root, x)
    start = (x - 2 * spacing) & M64
    others = [oracle.work_value(root, (start + k * spacing) & M64) for k in range(G) if k != 2]
    assert all(v < vx for v in others)
    r = eng.search(root, vx, start=start, device_mask=0, max_nonces_per_device=1)
    assert r.status == _lib.NPOW_OK and r.nonce == x and r.value == vx, (r, x)
    # 4. cancellation reaches every device
    tok = _lib.CancelToken()
    t = eng.submit(bytes(range(32)), M64, device_mask=0, cancel=tok)
    assert t.wait(0.2) is None
    tok.set()
    r = t.wait(30)
    assert r.status == _lib.NPOW_CANCELLED and r.nonces_done > 0
    # 5. a burst of jobs, each over every device
    roots = [bytes(rng.getrandbits(8) for _ in range(32)) for _ in range(48)]
    ts = [eng.submit(rt, LOW, start=rng.getrandbits(64), device_mask=0) for rt in roots]
    for rt, t in zip(roots, ts):
        r = t.wait(60)
        assert r.status == _lib.NPOW_OK and oracle.work_value(rt, r.nonce) == r.value >= LOW
    # 6. a sweep split over the devices is exact
    sroot = bytes(range(9, 41))
    hits = eng.sweep(sroot, 0xffff000000000000, 1 << 40, (1 << 22) + 13, device_mask=0)
    assert hits == oracle.sweep(sroot, 0xffff000000000000, 1 << 40, (1 << 22) + 13)
    # 6b. values through the shipped stream and per-lane pairs on the last device (a CU partition under
    #     NANOPOW_VIRTUAL_DEVICES: its grid is sized to its CUs, its copies stay on its own stream)
    vroot = bytes(range(70, 102))
    vals = eng.values(vroot, (1 << 40) - 1000, 4099, device=G - 1)
    assert vals == oracle.work_values([vroot] * 4099, [(1 << 40) - 1000 + i for i in range(4099)])
    pr = [bytes(rng.getrandbits(8) for _ in range(32)) for _ in range(257)]
    pn = [rng.getrandbits(64) for _ in range(257)]
    assert eng.values_pairs(pr, pn, device=G - 1) == oracle.work_values(pr, pn)
    # 7. a subset mask: devices 1 and 3 only
    for d in range(G):
        eng.reset_stats(d)
    r = eng.search(bytes(range(1, 33)), RECEIVE, device_mask=0b1010)
    assert r.status == _lib.NPOW_OK
    used = [eng.stats(d).launches > 0 for d in range(G)]
    assert used == [False, True, False, True], used
    out["affinity"] = [sum(eng.stats(d).affinity_checks for d in range(G)),
                       sum(eng.stats(d).affinity_failures for d in range(G))]
    out["ok"] = True
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
