"""Child process of tests/test_gpu_faults.py: the engine's GPU fault policy on one physical GPU
exposed as NANOPOW_VIRTUAL_DEVICES logical devices, with a fault injected through the engine's
test hooks (npow_pool.cpp header).  Reference: the work server drops a GPU that "returned invalid
work 3 consecutive times" and re-validates every GPU result on the CPU
(client/bin/windows/nano-work-server.exe @1669040, @1669144; SURVEY.md §5 failure recovery).

  invalid   NANOPOW_FAULT_INVALID=3, 8 devices: device 3's winners all read back corrupted.
            Every search still returns hashlib-valid work from the other devices; device 3 is
            dropped after exactly 3 invalid results and no search selects it afterwards.
  hip       NANOPOW_FAULT_HIP=2:3, 8 devices: device 2's 4th launch fails mid-job.  A bounded
            job whose only hit lies in the part of device 2's range it never reached still
            finds that hit (the remainder is re-strided onto the 7 survivors), device 2 is dead,
            later searches run on the survivors.
  exhaust   NANOPOW_FAULT_HIP=2:3, 8 devices: the same bounded job with no hit ends EXHAUSTED
            (not failed), nonces_done counting every nonce of the 8 ranges exactly once.
  allbad    NANOPOW_FAULT_INVALID=0,1, 2 devices: both devices only return invalid work; the
            search fails with NPOW_ERR_INVALID_WORK once the second one is dropped, and a new
            search has no device left (NPOW_ERR_NO_DEVICE).
  init      NANOPOW_FAULT_INIT=2, 4 devices: npow_init fails while opening device 2; a retry
            (hook removed) opens all 4 cleanly.
  cpu_last  NANOPOW_FAULT_HIP=0:0 and NANOPOW_TEST_CPU_RELEASE_DELAY_US, 1 GPU + 4 CPU worker threads:
            a bounded job over the GPU and the CPU device while a sweep holds the GPU; the CPU device hashes
            its range and its coordinator is held before it looks at the job; the GPU's first pool launch
            then fails, and its whole range goes to the CPU device, the only survivor.  The job must end
            EXHAUSTED with every nonce of both ranges hashed (nonces_done = 2 x the range), not released
            with the GPU's range unhashed.
  affinity  NANOPOW_TEST_AFFINITY_SKEW=1, 2 devices: device 1's pool worker finds its thread on the "wrong" HIP
            device at its first HIP call (the check's failure path, which a one-GPU box cannot reach otherwise):
            the call fails, device 1 is dropped, every search is still valid on device 0, and every HIP call
            site of device 0 was checked and found right.
  hooks_off NANOPOW_FAULT_INVALID=0,1 and NANOPOW_FAULT_INIT=0 WITHOUT NANOPOW_TEST_HOOKS=1, 2 devices:
            the hooks are ignored (a stray variable in a deployment must not drop GPUs): init
            succeeds, every search is valid, no device is dropped or counts an invalid result.

Prints one JSON line; exits non-zero on any mismatch."""
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
ITERS = 16                     # wave iterations per launch: a bounded job then spans several launches
PER_DEV = 20_000_000           # bounded job: nonces per device (5 launches of 4,194,304 at 4,096 waves)


def valid(root, r, thr):
    return r.status == _lib.NPOW_OK and oracle.work_value_hashlib(root, r.nonce) == r.value >= thr


def scenario_invalid(eng, G):
    rng = random.Random(11)
    n = 0
    while n < 400 and (n < 40 or not eng.stats(3).dead):  # device 3 wins ~1 search in 8 before it is dropped
        root = bytes(rng.getrandbits(8) for _ in range(32))
        r = eng.search(root, RECEIVE, start=rng.getrandbits(64), device_mask=0)
        assert valid(root, r, RECEIVE), r
        n += 1
    st = eng.stats(3)
    assert st.dead == 1 and st.invalid_work == 3, (st.dead, st.invalid_work)
    assert all(eng.stats(d).dead == 0 and eng.stats(d).invalid_work == 0 for d in range(G) if d != 3)
    # no search selects the dropped device any more
    try:
        eng.search(bytes(32), RECEIVE, device_mask=1 << 3)
        raise AssertionError("a search ran on the dropped device")
    except _lib.NanoPowError as e:
        assert e.code == _lib.NPOW_ERR_NO_DEVICE, e
    for d in range(G):
        eng.reset_stats(d)
    root = bytes(range(7, 39))
    r = eng.search(root, RECEIVE, device_mask=(1 << 3) | (1 << 5))
    assert valid(root, r, RECEIVE)
    assert eng.stats(3).launches == 0 and eng.stats(5).launches > 0
    return {"searches": n + 1, "device3_invalid": 3}


def bounded_setup(eng, G):
    """A root, start and threshold for which the union of the 8 bounded ranges
    [start + k*2^61, + PER_DEV) holds exactly one hit x, late in device 2's range (past what its
    first 3 launches cover).  Found with the GPU sweep (exact, tested against the oracle) and
    re-checked on the CPU."""
    spacing = (1 << 64) // G
    launch = 4096 * ITERS * 64
    for attempt in range(64):
        root = bytes([attempt]) + bytes(range(1, 32))
        start = (0x1234_5678_9abc << 8) + attempt
        base2 = (start + 2 * spacing) & M64
        lo = base2 + 3 * launch
        cand = eng.sweep(root, 0xffff000000000000, lo, base2 + PER_DEV - lo, device_mask=1, cap=1 << 12)
        if not cand:
            continue
        vals = {x: oracle.work_value(root, x) for x in cand}
        x = max(cand, key=lambda n: vals[n])
        vx = vals[x]
        union = []
        for k in range(G):
            union += eng.sweep(root, vx, (start + k * spacing) & M64, PER_DEV, device_mask=1, cap=16)
        if union == [x] and oracle.work_value_hashlib(root, x) == vx:
            return root, start, vx, x
    raise AssertionError("no suitable root")


def scenario_hip(eng, G):
    root, start, vx, x = bounded_setup(eng, G)
    eng.set_tuning(ITERS, 0, 0)
    r = eng.search(root, vx, start=start, device_mask=0, max_nonces_per_device=PER_DEV)
    assert r.status == _lib.NPOW_OK and r.nonce == x and r.value == vx, (r, hex(x))
    assert eng.stats(2).dead == 1
    rng = random.Random(5)
    for _ in range(16):  # the survivors keep serving
        rt = bytes(rng.getrandbits(8) for _ in range(32))
        rr = eng.search(rt, RECEIVE, start=rng.getrandbits(64), device_mask=0)
        assert valid(rt, rr, RECEIVE)
    return {"found_in_restrided_range": hex(x)}


def scenario_exhaust(eng, G):
    root, start, vx, x = bounded_setup(eng, G)
    eng.set_tuning(ITERS, 0, 0)
    r = eng.search(root, vx + 1, start=start, device_mask=0, max_nonces_per_device=PER_DEV)
    # device 2's done counters are never read back, but its bounded ranges are dense: the job counts
    # the ones whose launches completed there from their sizes, and the rest were re-strided onto the
    # survivors (hashed and counted once there) -- so every nonce of the 8 ranges is counted exactly once
    assert r.status == _lib.NPOW_EXHAUSTED and r.nonces_done == G * PER_DEV, (r, G * PER_DEV)
    assert eng.stats(2).dead == 1
    return {"nonces_done": r.nonces_done}


def scenario_allbad(eng, G):
    root = bytes(range(3, 35))
    try:
        eng.search(root, RECEIVE, device_mask=0)
        raise AssertionError("a search succeeded on devices that only return invalid work")
    except _lib.NanoPowError as e:
        assert e.code == _lib.NPOW_ERR_INVALID_WORK, e
    assert all(eng.stats(d).dead == 1 and eng.stats(d).invalid_work == 3 for d in range(G))
    try:
        eng.search(root, RECEIVE, device_mask=0)
        raise AssertionError("a search ran with every device dropped")
    except _lib.NanoPowError as e:
        assert e.code == _lib.NPOW_ERR_NO_DEVICE, e
    return {}


def scenario_init():
    """npow_init failing on device 2 of 4 leaves nothing behind: the retry opens 4 devices, ids
    0..3 in order, each serving its own searches (a partial init used to leave
    duplicate devices and leaked streams)."""
    try:
        _lib.Engine()
        raise AssertionError("npow_init ignored NANOPOW_FAULT_INIT")
    except _lib.NanoPowError as e:
        assert e.code == _lib.NPOW_ERR_HIP and "NANOPOW_FAULT_INIT" in e.message, e
    del os.environ["NANOPOW_FAULT_INIT"]
    eng = _lib.Engine()
    G = eng.n_devices
    assert G == 4, G
    rng = random.Random(9)
    for d in range(G):
        eng.reset_stats(d)
        rt = bytes(rng.getrandbits(8) for _ in range(32))
        r = eng.search(rt, RECEIVE, device_mask=1 << d)
        assert valid(rt, r, RECEIVE) and eng.stats(d).launches > 0
        assert all(eng.stats(k).launches == 0 for k in range(d + 1, G))
    return {"devices_after_retry": G}


def scenario_hooks_off(eng, G):
    rng = random.Random(21)
    for _ in range(24):
        root = bytes(rng.getrandbits(8) for _ in range(32))
        r = eng.search(root, RECEIVE, start=rng.getrandbits(64), device_mask=0)
        assert valid(root, r, RECEIVE), r
    assert all(eng.stats(d).dead == 0 and eng.stats(d).invalid_work == 0 for d in range(G))
    return {"searches": 24}


def scenario_cpu_last():
    import threading
    import time
    eng = _lib.Engine(cpu_threads=4)
    assert eng.n_devices == 2 and eng.cpu_device == 1, (eng.n_devices, eng.cpu_device)
    n = 1 << 20
    holder = threading.Thread(target=lambda: eng.sweep(bytes(range(32)), M64, 0, 1 << 34, device_mask=1))
    holder.start()  # the GPU is busy with a ~0.5-s sweep: the pool's GPU worker cannot launch meanwhile
    time.sleep(0.05)
    t0 = time.perf_counter()
    r = eng.search(bytes(range(5, 37)), M64, start=1 << 44, device_mask=0b11, max_nonces_per_device=n)
    dt = time.perf_counter() - t0
    holder.join()
    assert eng.stats(0).dead == 1, "the GPU's injected launch failure did not drop it"
    assert r.status == _lib.NPOW_EXHAUSTED and r.nonces_done == 2 * n, (r, 2 * n)
    assert eng.stats(1).nonces == 2 * n, eng.stats(1).nonces  # both ranges hashed on the CPU device, counted as hashed
    return {"nonces_done": r.nonces_done, "seconds": round(dt, 3), "devices": 2}


def scenario_affinity(eng, G):
    rng = random.Random(31)
    for _ in range(24):
        root = bytes(rng.getrandbits(8) for _ in range(32))
        r = eng.search(root, RECEIVE, start=rng.getrandbits(64), device_mask=0)
        assert valid(root, r, RECEIVE), r
    s0, s1 = eng.stats(0), eng.stats(1)
    assert s1.dead == 1 and s1.affinity_failures >= 1, (s1.dead, s1.affinity_failures)
    assert s0.dead == 0 and s0.affinity_checks > 0 and s0.affinity_failures == 0, (s0.affinity_checks,
                                                                                s0.affinity_failures)
    return {"device0_checks": s0.affinity_checks, "device1_failures": s1.affinity_failures}


def main():
    which = sys.argv[1]
    if which == "cpu_last":
        out = scenario_cpu_last()
        out.update({"scenario": which, "ok": True})
        print(json.dumps(out), flush=True)
        return
    if which == "init":
        out = scenario_init()
        out.update({"scenario": which, "devices": 4, "ok": True})
        print(json.dumps(out), flush=True)
        return
    eng = _lib.Engine()
    G = eng.n_devices
    assert G == int(os.environ["NANOPOW_VIRTUAL_DEVICES"]), G
    fn = {"invalid": scenario_invalid, "hip": scenario_hip, "exhaust": scenario_exhaust,
          "allbad": scenario_allbad, "hooks_off": scenario_hooks_off, "affinity": scenario_affinity}[which]
    out = fn(eng, G)
    out.update({"scenario": which, "devices": G, "ok": True})
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
