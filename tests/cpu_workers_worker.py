"""Child process of tests/test_gpu_pool.py::test_cpu_workers_beside_the_gpu: the work pool's CPU workers
(nano-work-server.exe @1681064 `--cpu-threads`; npow_config_cpu_threads, nano-dpow_amd/csrc/npow_cpu.cpp)
beside the GPU(s).  CPU workers must be configured before npow_init, which is process-wide, hence a
process of its own.  Every result is checked with hashlib (oracle.work_value_hashlib).  Prints one JSON
line; exits non-zero on any mismatch."""
import json
import os
import random
import statistics
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(ROOT, "nano-dpow_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import oracle  # noqa: E402  (the checker)
from nanopow import _lib  # noqa: E402

M64 = (1 << 64) - 1
RECEIVE, EASY = 0xfffffe0000000000, 0xfff0000000000000
THREADS = 4


def main():
    eng = _lib.Engine(cpu_threads=THREADS)
    G = eng.n_devices
    cpu = eng.cpu_device
    assert cpu == G - 1, (cpu, G)
    st = eng.stats(cpu)
    assert st.hip_device == -1 and st.cus == THREADS and st.grid == 0, (st.hip_device, st.cus, st.grid)
    assert all(eng.stats(d).hip_device >= 0 for d in range(G - 1))
    assert eng.gpu_mask == (1 << (G - 1)) - 1
    out = {"devices": G, "cpu_device": cpu}
    rng = random.Random(5)
    cmask = 1 << cpu
    # 1. searches on the CPU workers alone (p = 2^-12 per nonce): valid, decided by the CPU device
    for _ in range(8):
        root = bytes(rng.getrandbits(8) for _ in range(32))
        t = eng.submit(root, EASY, start=rng.getrandbits(64), device_mask=cmask)
        info = t.wait_info(60)
        assert info.status == _lib.NPOW_OK and info.winner_device == cpu, (info.status, info.winner_device)
        assert oracle.work_value_hashlib(root, info.nonce) == info.value >= EASY
    # 2. bounded exhaustion on the CPU: exactly the range, counted exactly
    eng.reset_stats(cpu)
    r = eng.search(bytes(32), M64, start=12345, device_mask=cmask, max_nonces_per_device=100_003)
    assert r.status == _lib.NPOW_EXHAUSTED and r.nonces_done == 100_003, r
    assert eng.stats(cpu).nonces == 100_003
    # 2b. a bounded search over all devices (mask 0) leaves the CPU workers out: the GPUs exhaust
    #     their ranges alone, at GPU speed; naming the CPU device explicitly still includes it (and takes far longer)
    n_b = 1 << 20
    t_gpu, t_all = [], []
    for i in range(3):
        before = eng.stats(cpu).launches
        t0 = time.perf_counter()
        r = eng.search(bytes(32), M64, start=i << 50, device_mask=0, max_nonces_per_device=n_b)
        t_gpu.append(time.perf_counter() - t0)
        assert r.status == _lib.NPOW_EXHAUSTED and r.nonces_done == (G - 1) * n_b, r
        assert eng.stats(cpu).launches == before, "a bounded mask-0 search used the CPU device"
        t0 = time.perf_counter()
        r = eng.search(bytes(32), M64, start=i << 50, device_mask=(1 << G) - 1, max_nonces_per_device=n_b)
        t_all.append(time.perf_counter() - t0)
        assert r.status == _lib.NPOW_EXHAUSTED and r.nonces_done == G * n_b, r
    out["bounded_exhaust_ms"] = {"mask0_gpus_only": round(statistics.median(t_gpu) * 1e3, 3),
                                 "with_cpu_device": round(statistics.median(t_all) * 1e3, 3)}
    assert statistics.median(t_gpu) < statistics.median(t_all), out
    # 3. a range smaller than one claim is hashed in order by one thread: the first hit is returned
    root = bytes(range(40, 72))
    start = 1 << 50
    vals = oracle.work_values([root] * 5000, [start + i for i in range(5000)])
    first = next(i for i, v in enumerate(vals) if v >= EASY)
    r = eng.search(root, EASY, start=start, device_mask=cmask, max_nonces_per_device=5000)
    assert r.status == _lib.NPOW_OK and r.nonce == start + first and r.value == vals[first], (r, first)
    # 4. the only hit lies in the CPU device's stride of a GPU + CPU job (device k of G starts at
    #    start + k * 2^64 / G): the CPU device decides it; the GPUs exhaust their bounded ranges
    spacing = (1 << 64) // G
    n = 3000
    base = rng.getrandbits(64)
    cpu_vals = oracle.work_values([root] * n, [(base + cpu * spacing + i) & M64 for i in range(n)])
    best = max(range(n), key=lambda i: cpu_vals[i])
    thr = cpu_vals[best]
    gpu_best = max(max(oracle.work_values([root] * n, [(base + k * spacing + i) & M64 for i in range(n)]))
                   for k in range(G - 1))
    assert gpu_best < thr
    t = eng.submit(root, thr, start=base, device_mask=(1 << G) - 1, max_nonces_per_device=n)  # (mask 0 would
    info = t.wait_info(60)                                           # leave the CPU out of a bounded search: 2b)
    assert info.status == _lib.NPOW_OK and info.winner_device == cpu, (info.status, info.winner_device)
    assert info.nonce == (base + cpu * spacing + best) & M64 and info.value == thr
    # 5. GPU + CPU at receive difficulty: valid work; the CPU device takes part; GPU-won jobs are not
    #    held up by it (it reads the decision every 256 nonces and is released within ~0.1 ms)
    for d in range(G):
        eng.reset_stats(d)
    ttw, winners = [], []
    for _ in range(60):
        root = bytes(rng.getrandbits(8) for _ in range(32))
        t0 = time.perf_counter()
        t = eng.submit(root, RECEIVE, start=rng.getrandbits(64), device_mask=0)
        info = t.wait_info(60)
        ttw.append((time.perf_counter() - t0) * 1e3)
        assert info.status == _lib.NPOW_OK and oracle.work_value_hashlib(root, info.nonce) == info.value >= RECEIVE
        assert info.n_devices == G
        winners.append(info.winner_device)
    cpu_n = eng.stats(cpu).nonces
    assert cpu_n > 0
    out["mixed_receive"] = {"p50_ms": round(statistics.median(ttw), 3), "max_ms": round(max(ttw), 3),
                            "cpu_nonces": cpu_n, "gpu_nonces": sum(eng.stats(d).nonces for d in range(G - 1)),
                            "cpu_wins": winners.count(cpu)}
    assert statistics.median(ttw) < 5.0, out
    # 6. cancellation reaches the CPU workers
    tok = _lib.CancelToken()
    t = eng.submit(bytes(range(32)), M64, device_mask=cmask, cancel=tok)
    assert t.wait(0.2) is None
    tok.set()
    r = t.wait(10)
    assert r.status == _lib.NPOW_CANCELLED and r.nonces_done > 0
    # 7. sweeps and values run on the GPUs only: mask 0 is exact, the CPU device alone is refused
    sroot = bytes(range(9, 41))
    hits = eng.sweep(sroot, 0xffff000000000000, 1 << 40, (1 << 20) + 7, device_mask=0)
    assert hits == oracle.sweep(sroot, 0xffff000000000000, 1 << 40, (1 << 20) + 7)
    try:
        eng.sweep(sroot, 0xffff000000000000, 0, 1 << 16, device_mask=cmask)
        raise AssertionError("a sweep on the CPU device alone must be refused")
    except _lib.NanoPowError as e:
        assert e.code == _lib.NPOW_ERR_NO_DEVICE
    try:
        eng.values(sroot, 0, 16, device=cpu)
        raise AssertionError("values on the CPU device must be refused")
    except _lib.NanoPowError as e:
        assert e.code == _lib.NPOW_ERR_BAD_ARGUMENT
    st = eng.stats(cpu)
    out["cpu_rate_mnps"] = round(st.nonces / max(st.kernel_ms, 1e-9) / 1e3, 2)
    # 8. the CPU device's rate alone and beside an endless GPU search (the win watcher spun a core for as
    #    long as a GPU slot was armed, next to the CPU hashing threads): recorded, not asserted (a timing)
    def cpu_rate(with_gpu):
        gtok = _lib.CancelToken()
        g = eng.submit(bytes(range(50, 82)), M64, device_mask=1, cancel=gtok) if with_gpu else None
        time.sleep(0.05)
        eng.reset_stats(cpu)
        ctok = _lib.CancelToken()
        c = eng.submit(bytes(range(60, 92)), M64, device_mask=cmask, cancel=ctok)
        time.sleep(0.5)
        ctok.set()
        c.wait(10)
        s2 = eng.stats(cpu)
        if g is not None:
            gtok.set()
            g.wait(10)
        return s2.nonces / max(s2.kernel_ms, 1e-9) / 1e3
    alone, beside = cpu_rate(False), cpu_rate(True)
    out["cpu_rate_alone_vs_beside_gpu_mnps"] = [round(alone, 2), round(beside, 2), round(beside / max(alone, 1e-9), 3)]
    out["ok"] = True
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
