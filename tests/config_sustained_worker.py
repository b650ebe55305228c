"""Child process of tests/test_gpu_configs.py for BASELINE configs[4] ("Sustained node throughput
at epoch-2 send difficulty with per-GPU nonce striding"): NANOPOW_VIRTUAL_DEVICES logical devices,
every search split over all of them (device k from start + k * 2^64 / G).

1. single-search rate: one search at a time (npow_search over every device), SINGLE_S seconds;
2. sustained: SUSTAINED_S seconds of fresh roots through the work pool (npow_submit), DEPTH
   searches in flight per device, every reply re-validated with hashlib.

Prints one JSON line: both rates (nonces hashed / wall time), search counts, invalid replies."""
import hashlib
import json
import os
import sys
import time
from collections import deque

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "nano-dpow_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "oracle"))

import oracle  # noqa: E402  (the checker)
from nanopow import _lib  # noqa: E402

SEND = 0xfffffff800000000


def root_of(i: int) -> bytes:
    return hashlib.blake2b(b"sustained" + i.to_bytes(8, "little"), digest_size=32).digest()


def main():
    single_s = float(os.environ.get("SINGLE_S", "8"))
    sustained_s = float(os.environ.get("SUSTAINED_S", "60"))
    depth = int(os.environ.get("DEPTH", "4"))
    eng = _lib.Engine()
    G = eng.n_devices
    for i in range(3):  # warm up every device's worker and kernels
        eng.search(root_of(10_000_000 + i), SEND, device_mask=0)
    bad = 0
    # 1. one search at a time over every device
    t0 = time.perf_counter()
    n1 = nonces1 = 0
    while time.perf_counter() - t0 < single_s:
        rt = root_of(n1)
        r = eng.search(rt, SEND, start=n1 << 40, device_mask=0)
        bad += r.status != _lib.NPOW_OK or oracle.work_value_hashlib(rt, r.nonce) != r.value or r.value < SEND
        nonces1 += r.nonces_done
        n1 += 1
    single = nonces1 / (time.perf_counter() - t0) / 1e9
    # 2. sustained: depth x G searches in flight, fresh roots, every reply re-validated
    pending = deque()
    nxt = 1_000_000
    n2 = nonces2 = 0
    t0 = time.perf_counter()
    while True:
        now = time.perf_counter()
        while len(pending) < depth * G and now - t0 < sustained_s:
            rt = root_of(nxt)
            pending.append((rt, eng.submit(rt, SEND, start=nxt << 40, device_mask=0)))
            nxt += 1
        if not pending:
            break
        rt, t = pending.popleft()
        r = t.wait()
        bad += r.status != _lib.NPOW_OK or oracle.work_value_hashlib(rt, r.nonce) != r.value or r.value < SEND
        nonces2 += r.nonces_done
        n2 += 1
    wall2 = time.perf_counter() - t0
    sustained = nonces2 / wall2 / 1e9
    print(json.dumps({"devices": G, "single_gnps": round(single, 4), "single_searches": n1,
                      "sustained_gnps": round(sustained, 4), "sustained_searches": n2, "sustained_s": round(wall2, 2),
                      "depth_per_device": depth, "invalid": int(bad),
                      "ratio": round(sustained / single, 4)}), flush=True)


if __name__ == "__main__":
    main()
