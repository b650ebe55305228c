"""Child process of tests/test_gpu_kernels.py: the shipped search / sweep kernels (four 512-lane
workgroups per CU: npow_pool_kernel_ls2*, npow_sweep_kernel_ls2), checked end to end
against the oracle in a fresh process.

It runs: 24 first-win searches at receive difficulty (every result re-hashed by hashlib), 8
concurrent searches (one launch table with several entries), a bounded search with no hit that
must end EXHAUSTED after exactly its nonce budget (the dense bounded mapping: a wrong mapping
hashes some nonces twice and others never), a bounded search whose only hit lies near the end of
its range, and an exhaustive 2^26 sweep whose hit set must equal the oracle's.  Prints one JSON line.
"""
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
RECEIVE = 0xfffffe0000000000
LOW = 0xffff000000000000


def main(variant):
    eng = _lib.Engine()
    rng = random.Random(1)
    for _ in range(24):
        root = bytes(rng.getrandbits(8) for _ in range(32))
        r = eng.search(root, RECEIVE, start=rng.getrandbits(64), device_mask=1)
        assert r.status == _lib.NPOW_OK and oracle.work_value_hashlib(root, r.nonce) == r.value >= RECEIVE, r
    roots = [bytes(rng.getrandbits(8) for _ in range(32)) for _ in range(8)]
    tickets = [eng.submit(rt, RECEIVE, start=rng.getrandbits(64), device_mask=1) for rt in roots]
    for rt, t in zip(roots, tickets):
        r = t.wait(30)
        assert r.status == _lib.NPOW_OK and oracle.work_value_hashlib(rt, r.nonce) == r.value >= RECEIVE, r
    # bounded, no hit possible (threshold 2^64-1 is met by nonces whose value is all ones only)
    count = 3 * (1 << 22) + 12345
    r = eng.search(bytes(range(32)), M64, start=1 << 40, device_mask=1, max_nonces_per_device=count)
    assert r.status == _lib.NPOW_EXHAUSTED and r.nonces_done == count, (r.status, r.nonces_done, count)
    # bounded, the range's only hit at LOW is its last nonce: found, and it is the oracle's
    root = bytes(rng.getrandbits(8) for _ in range(32))
    hits = oracle.sweep(root, LOW, 0, 1 << 22, threads=16)
    assert len(hits) >= 2, "too few hits in [0, 2^22) for the probe root"
    first, last = hits[-2] + 1, hits[-1]
    r = eng.search(root, LOW, start=first, device_mask=1, max_nonces_per_device=last - first + 1)
    assert r.status == _lib.NPOW_OK and r.nonce == last and oracle.work_value_hashlib(root, r.nonce) == r.value, r
    # exhaustive sweep, exact hit set
    root = bytes(rng.getrandbits(8) for _ in range(32))
    got = eng.sweep(root, LOW, 5, 1 << 26, device_mask=1)
    want = oracle.sweep(root, LOW, 5, 1 << 26, threads=16)
    assert got == want, (len(got), len(want))
    print(json.dumps({"variant": variant, "ok": True, "sweep_hits": len(got),
                      "pool_groups": int(eng.stats(0).pool_groups)}))


if __name__ == "__main__":
    main(sys.argv[1])
