#!/usr/bin/env python3
"""Round-5 probe: serial searches then a sweep, timed, NANOPOW_DEBUG's timestamped pool log beside (stderr).
    NANOPOW_DEBUG=1 python3 tools/experiments/linger_probe.py ROUNDS 2> log"""
import os
import random
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "nano-dpow_amd"))
import nanopow  # noqa: E402

eng = nanopow.engine()
rng = random.Random(5)
for rnd in range(int(sys.argv[1])):
    n = 300 if rnd == 0 else 3
    for i in range(n):
        r = bytes(rng.getrandbits(8) for _ in range(32))
        res = eng.submit(r, 0xfffffe0000000000, start=i << 40, device_mask=1).wait(30)
        assert res.status == 0
    t = time.perf_counter()
    print(f"[{time.monotonic() * 1e3:.3f}] probe: sweep start", file=sys.stderr, flush=True)
    eng.sweep(r, 0xffffffc000000000, 0, 1 << 22, device_mask=1)
    dt = time.perf_counter() - t
    print(f"[{time.monotonic() * 1e3:.3f}] probe: sweep end {dt * 1e3:.2f} ms", file=sys.stderr, flush=True)
    print(f"round {rnd}: sweep {dt * 1e3:.2f} ms", flush=True)
