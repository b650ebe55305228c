#!/usr/bin/env python3
"""Soak test of the work pool on the GPU: a random mix of concurrent work for --seconds,
every result checked.  Prints a progress line every 10 s and one JSON summary line; exits
non-zero on the first wrong result.

Mix (per client thread, chosen at random each round):
  * unbounded searches at thresholds between fffff000... and fffffff8...; winners must
    re-validate on the CPU (npow_work_value) at their own threshold;
  * the same, cancelled by token or by ticket at a random time, or abandoned (ticket dropped);
  * bounded no-hit ranges (threshold 2^64-1) of ragged lengths: EXHAUSTED after exactly
    that many nonces;
  * small exact sweeps checked against the C oracle;
  * max_active and launch-budget changes from a separate thread (yields, queueing).

With --faults (run with NANOPOW_VIRTUAL_DEVICES and NANOPOW_FAULT_INVALID, npow_pool.cpp): bounded
ranges run over every device too, and must end EXHAUSTED having hashed at least n nonces per device
alive when they were submitted, less one device (a device dropped mid-job hands what it had not
finished to the others, which may hash part of it again); searches must still all succeed.

Usage (GPU box): python3 tools/pool_soak.py [--seconds 180] [--clients 24] [--faults]
"""
import argparse
import json
import os
import random
import sys
import threading
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(ROOT, "nano-dpow_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import oracle  # noqa: E402  (the checker)
from nanopow import _lib  # noqa: E402

M64 = (1 << 64) - 1


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=180.0)
    ap.add_argument("--clients", type=int, default=24)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--faults", action="store_true", help="a fault hook is set: bounded ranges over every device")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="CPU workers beside the GPU(s) (npow_config_cpu_threads): every mask-0 search also runs on them")
    args = ap.parse_args()
    eng = _lib.Engine(cpu_threads=args.cpu_threads)
    stop = time.time() + args.seconds
    counts = {"search": 0, "cancel_token": 0, "cancel_ticket": 0, "abandoned": 0, "bounded": 0, "sweep": 0,
              "reconfig": 0}
    lock = threading.Lock()
    errors = []

    def bump(k):
        with lock:
            counts[k] += 1

    def fail(msg):
        with lock:
            errors.append(msg)

    def client(cid):
        rng = random.Random(args.seed * 1000 + cid)
        while time.time() < stop and not errors:
            root = bytes(rng.getrandbits(8) for _ in range(32))
            kind = rng.random()
            try:
                if kind < 0.45:
                    thr = rng.choice([0xfffff00000000000, 0xfffffe0000000000, 0xffffff0000000000, 0xfffffff800000000])
                    t = eng.submit(root, thr, start=rng.getrandbits(64))
                    early = t.wait_result(120) if rng.random() < 0.5 else None  # the outcome at the decision
                    r = t.wait(120)
                    if r is None or r.status != _lib.NPOW_OK or eng.work_value(root, r.nonce) != r.value or r.value < thr:
                        fail(f"search {root.hex()} {thr:016x}: {r}")
                    if early is not None and (early.status, early.nonce, early.value) != (r.status, r.nonce, r.value):
                        fail(f"wait_result {early} differs from wait {r}")
                    bump("search")
                elif kind < 0.65:
                    tok = _lib.CancelToken()
                    t = eng.submit(root, M64, start=rng.getrandbits(64), cancel=tok)
                    time.sleep(rng.uniform(0, 0.05))
                    how = rng.random()
                    if how < 0.4:
                        tok.set()
                        bump("cancel_token")
                    elif how < 0.8:
                        t.cancel()
                        bump("cancel_ticket")
                    else:
                        del t  # abandoned: the finaliser cancels and collects it
                        bump("abandoned")
                        continue
                    r = t.wait(30)
                    if r is None or r.status != _lib.NPOW_CANCELLED:
                        fail(f"cancel {root.hex()}: {r}")
                elif kind < 0.85:
                    n = rng.choice([1, 63, 64, 65, 1000, 4097, 1 << 16, (1 << 20) + 3, 1 << 24])
                    if args.faults:
                        alive = sum(1 for d in range(eng.n_devices) if not eng.stats(d).dead)
                        r = eng.submit(root, M64, start=rng.getrandbits(64), device_mask=0,
                                       max_nonces_per_device=n).wait(120)
                        if r is None or r.status != _lib.NPOW_EXHAUSTED or r.nonces_done < n * (alive - 1):
                            fail(f"bounded {n} over {alive} devices: {r}")
                    else:
                        r = eng.submit(root, M64, start=rng.getrandbits(64), device_mask=1,
                                       max_nonces_per_device=n).wait(120)
                        if r is None or r.status != _lib.NPOW_EXHAUSTED or r.nonces_done != n:
                            fail(f"bounded {n}: {r}")
                    bump("bounded")
                else:
                    start, cnt = rng.getrandbits(64), rng.choice([1000, 65536, 1 << 20])
                    thr = 0xfff0000000000000
                    got = eng.sweep(root, thr, start, cnt, device_mask=1, cap=1 << 12)
                    want = oracle.sweep(root, thr, start, cnt, threads=2)
                    if got != want:
                        fail(f"sweep {root.hex()} {start} {cnt}: {len(got)} vs {len(want)}")
                    bump("sweep")
            except Exception as e:  # noqa: BLE001
                fail(f"client {cid}: {type(e).__name__}: {e}")

    def reconfig():
        rng = random.Random(args.seed)
        while time.time() < stop and not errors:
            time.sleep(rng.uniform(0.5, 3.0))
            eng.pool_config(rng.choice([1, 4, 16, 64]))
            eng.set_pool_tuning(budget_us=rng.choice([5_000, 20_000, 100_000]))
            bump("reconfig")
        eng.pool_config(64)
        eng.set_pool_tuning(budget_us=20_000)

    ths = [threading.Thread(target=client, args=(i,), daemon=True) for i in range(args.clients)]
    ths.append(threading.Thread(target=reconfig, daemon=True))
    t0 = time.time()
    for t in ths:
        t.start()
    last = t0
    while any(t.is_alive() for t in ths):
        time.sleep(0.5)
        if time.time() - last >= 10:
            last = time.time()
            with lock:
                print(f"[soak] {last - t0:.0f}s {counts} errors={len(errors)}", flush=True)
        if errors:
            break
    for t in ths:
        t.join(120)
    st = eng.stats(0)
    out = {"seconds": round(time.time() - t0, 1), "clients": args.clients, "counts": counts,
           "errors": errors[:5], "pool_status_end": list(eng.pool_status()), "device0_nonces": st.nonces,
           "invalid_work": [eng.stats(d).invalid_work for d in range(eng.n_devices)],
           "dead": [eng.stats(d).dead for d in range(eng.n_devices)]}
    print(json.dumps(out), flush=True)
    return 1 if errors or tuple(eng.pool_status()) != (0, 0) else 0


if __name__ == "__main__":
    sys.exit(main())
