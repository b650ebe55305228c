#!/usr/bin/env python3
"""Round-5 probe of lingering launches: serial searches (each split over every device of the mask), optionally a
sweep after each round, timed; NANOPOW_DEBUG's timestamped pool log beside it on stderr (lingering launch ended ->
launch done: how long a yielded lingering launch takes to end).
    NANOPOW_DEBUG=1 python3 tools/experiments/linger_probe.py ROUNDS SEARCHES_PER_ROUND [sweep] 2> log"""
import os
import random
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "nano-dpow_amd"))
import nanopow  # noqa: E402

eng = nanopow.engine()
mask = (1 << eng.n_devices) - 1
rng = random.Random(5)
rounds, per = int(sys.argv[1]), int(sys.argv[2])
sweep = len(sys.argv) > 3 and sys.argv[3] == "sweep"
for rnd in range(rounds):
    t0 = time.perf_counter()
    for i in range(per):
        r = bytes(rng.getrandbits(8) for _ in range(32))
        res = eng.submit(r, 0xfffffe0000000000, start=i << 40, device_mask=mask).wait(30)
        assert res.status == 0
    dt_s = time.perf_counter() - t0
    msg = f"round {rnd}: {per} searches {dt_s * 1e3:.2f} ms"
    if sweep:
        t = time.perf_counter()
        print(f"[{time.monotonic() * 1e3:.3f}] probe: sweep start", file=sys.stderr, flush=True)
        eng.sweep(r, 0xffffffc000000000, 0, 1 << 22, device_mask=1)
        dt = time.perf_counter() - t
        print(f"[{time.monotonic() * 1e3:.3f}] probe: sweep end {dt * 1e3:.2f} ms", file=sys.stderr, flush=True)
        msg += f", sweep {dt * 1e3:.2f} ms"
    print(msg, flush=True)
