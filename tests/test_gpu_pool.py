"""GPU work pool (npow_submit / npow_wait / npow_cancel; npow_pool_kernel): many roots per launch.

Bit-exact against the oracle throughout: every winner re-validates under hashlib at its own
threshold, every bounded range without a hit is reported EXHAUSTED with exactly its nonce
count hashed, every bounded range with hits returns one of the fixture's hits, and the
nonces the jobs report add up to the device's own counter.  Run on an MI355X: ``pytest -m gpu``.
"""
import random
import time

import pytest

import oracle
from conftest import load_golden
from nanopow import _lib

pytestmark = pytest.mark.gpu
M64 = (1 << 64) - 1
SEND, RECEIVE, LOW = 0xfffffff800000000, 0xfffffe0000000000, 0xfffff00000000000


def _roots(seed, n):
    rng = random.Random(seed)
    return [bytes(rng.getrandbits(8) for _ in range(32)) for _ in range(n)]


def test_many_roots_in_flight_all_revalidate(gpu_engine):
    """200 roots at three thresholds submitted at once: up to 64 share each launch."""
    roots = _roots(11, 200)
    thr = [LOW, RECEIVE, 0xffffc00000000000]
    tickets = [gpu_engine.submit(r, thr[i % 3], start=i << 48) for i, r in enumerate(roots)]
    for i, (r, t) in enumerate(zip(roots, tickets)):
        res = t.wait(60)
        assert res is not None and res.status == _lib.NPOW_OK, i
        assert oracle.work_value_hashlib(r, res.nonce) == res.value >= thr[i % 3]
        assert res.nonces_done > 0


def test_nonce_accounting_matches_device_counter(gpu_engine):
    """Jobs that win, are cancelled, and keep running side by side (waves migrate between
    them): the nonces each job reports sum to what the device counted."""
    gpu_engine.reset_stats(0)
    roots = _roots(12, 40)
    toks = [_lib.CancelToken() for _ in range(8)]
    never = [gpu_engine.submit(r, M64, start=7 << 50, device_mask=1, cancel=c) for r, c in zip(roots[:8], toks)]
    quick = [gpu_engine.submit(r, LOW, device_mask=1) for r in roots[8:]]
    done = 0
    for r, t in zip(roots[8:], quick):
        res = t.wait(60)
        assert res.status == _lib.NPOW_OK and oracle.work_value(r, res.nonce) == res.value >= LOW
        done += res.nonces_done
    time.sleep(0.05)
    for c in toks:
        c.set()
    for t in never:
        res = t.wait(30)
        assert res.status == _lib.NPOW_CANCELLED and res.nonces_done > 0
        done += res.nonces_done
    st = gpu_engine.stats(0)
    assert st.nonces == done
    # the quick jobs shared launches with the endless ones: most finished from the kernel's published
    # final count, before their launch ended (npow_kernel.hip "Early finish"), and every such count
    # equals the read-back after the launch
    assert st.early_finishes >= 16 and st.early_mismatches == 0, (st.early_finishes, st.early_mismatches)


def test_bounded_ranges_exact_beside_unbounded_jobs(gpu_engine):
    """Bounded ranges (max_nonces) are covered exactly once even while unbounded jobs in the
    same launches hand waves around: gaps between consecutive fixture hits are EXHAUSTED
    after exactly gap nonces; ranges that hold hits return one of them."""
    c = load_golden("sweeps_small.json")["cases"][1]  # RECEIVE hits of root 0 in [0, 2^28)
    root, thr = bytes.fromhex(c["root"]), int(c["threshold"], 16)
    hits = [int(h, 16) for h in c["hits"]]
    tok = _lib.CancelToken()
    busy = [gpu_engine.submit(r, M64, device_mask=1, cancel=tok) for r in _roots(13, 4)]
    gaps = [(hits[i] + 1, hits[i + 1] - hits[i] - 1) for i in range(min(12, len(hits) - 1))]
    gap_t = [gpu_engine.submit(root, thr, start=s, device_mask=1, max_nonces_per_device=n) for s, n in gaps]
    span_t = [gpu_engine.submit(root, thr, start=hits[i] - 5, device_mask=1, max_nonces_per_device=1000)
              for i in range(4)]
    for (s, n), t in zip(gaps, gap_t):
        res = t.wait(60)
        assert res.status == _lib.NPOW_EXHAUSTED and res.nonce is None
        assert res.nonces_done == n
    for i, t in enumerate(span_t):
        res = t.wait(60)
        assert res.status == _lib.NPOW_OK and res.nonce == hits[i]  # the only hit in its range
    tok.set()
    for t in busy:
        assert t.wait(30).status == _lib.NPOW_CANCELLED


def test_wait_timeout_and_ticket_cancel(gpu_engine):
    t = gpu_engine.submit(bytes(32), M64, device_mask=1)
    assert t.wait(0.01) is None
    q, a = gpu_engine.pool_status()
    assert a >= 1
    t.cancel()
    res = t.wait(10)
    assert res.status == _lib.NPOW_CANCELLED and res.nonces_done > 0


def test_max_active_queues_the_rest(gpu_engine):
    gpu_engine.pool_config(2)
    try:
        toks = [_lib.CancelToken() for _ in range(5)]
        ts = [gpu_engine.submit(r, M64, device_mask=1, cancel=c) for r, c in zip(_roots(14, 5), toks)]
        time.sleep(0.05)
        assert gpu_engine.pool_status() == (3, 2)
        toks[4].set()  # a queued job cancelled before it ever ran
        res = ts[4].wait(10)
        assert res.status == _lib.NPOW_CANCELLED and res.nonces_done == 0
        for c in toks[:4]:
            c.set()
        for t in ts[:4]:
            assert t.wait(30).status == _lib.NPOW_CANCELLED
    finally:
        gpu_engine.pool_config(64)
    assert gpu_engine.pool_status() == (0, 0)


def test_sweep_waits_for_the_device_and_both_finish(gpu_engine):
    root = bytes(range(3, 35))
    tickets = [gpu_engine.submit(r, RECEIVE, device_mask=1) for r in _roots(15, 8)]
    hits = gpu_engine.sweep(root, 0xffff000000000000, 0, 1 << 22, device_mask=1)
    assert hits == oracle.sweep(root, 0xffff000000000000, 0, 1 << 22)
    for t in tickets:
        assert t.wait(60).status == _lib.NPOW_OK


def test_batch_of_64_with_cancels(gpu_engine):
    roots = _roots(16, 64)
    thr = [RECEIVE] * 48 + [M64] * 16
    toks = [None] * 48 + [_lib.CancelToken() for _ in range(16)]
    for c in toks[48:]:
        c.set()
    res, done = gpu_engine.search_batch(roots, thr, cancels=toks)
    for r, x in zip(roots[:48], res[:48]):
        assert x.status == _lib.NPOW_OK and oracle.work_value(r, x.nonce) == x.value >= RECEIVE
    assert all(x.status == _lib.NPOW_CANCELLED for x in res[48:])
    assert done > 0


@pytest.mark.parametrize("count", [1, 63, 64, 65, 4095, (1 << 20) + 7])
def test_bounded_ragged_counts_exhaust_exactly(gpu_engine, count):
    """Ragged bounded ranges (partial last block, fewer blocks than waves) are hashed exactly
    once, including a range that wraps 2^64 -> 0; several of them share the launch."""
    starts = [0, 12345, M64 - count // 2]
    ts = [gpu_engine.submit(bytes(range(32)), M64, start=s, device_mask=1, max_nonces_per_device=count)
          for s in starts]
    for t in ts:
        r = t.wait(60)
        assert r.status == _lib.NPOW_EXHAUSTED and r.nonces_done == count


def test_bounded_first_hit_in_ragged_ranges(gpu_engine):
    """Threshold 0 makes every nonce a hit: the winner of a bounded range must lie inside it,
    for ragged lengths and a range across 2^64; an exact-value threshold finds exactly that nonce."""
    root = bytes(range(7, 39))
    for start, count in [(M64 - 2, 5), (1000, 1), (77, 65)]:
        r = gpu_engine.submit(root, 0, start=start, device_mask=1, max_nonces_per_device=count).wait(60)
        assert r.status == _lib.NPOW_OK
        assert (r.nonce - start) & M64 < count and r.value == oracle.work_value(root, r.nonce)
    vals = gpu_engine.values(root, 5000, 3000)
    top = max(range(3000), key=lambda i: vals[i])
    r = gpu_engine.submit(root, vals[top], start=5000, device_mask=1, max_nonces_per_device=3000).wait(60)
    assert r.status == _lib.NPOW_OK and r.nonce == 5000 + top and r.value == vals[top]
    r = gpu_engine.submit(root, vals[top] + 1, start=5000, device_mask=1, max_nonces_per_device=3000).wait(60)
    assert r.status == _lib.NPOW_EXHAUSTED and r.nonces_done == 3000


def test_duplicate_roots_in_flight_are_independent_jobs(gpu_engine):
    """The same root submitted several times at once (a collision in the burst): every ticket
    gets its own valid answer; cancelling one leaves the others running to completion."""
    root = bytes(range(100, 132))
    toks = [_lib.CancelToken() for _ in range(6)]
    ts = [gpu_engine.submit(root, RECEIVE, start=i << 58, device_mask=1, cancel=toks[i]) for i in range(6)]
    toks[2].set()
    for i, t in enumerate(ts):
        r = t.wait(60)
        if i == 2 and r.status == _lib.NPOW_CANCELLED:
            continue
        assert r.status == _lib.NPOW_OK and oracle.work_value(root, r.nonce) == r.value >= RECEIVE


def test_full_table_of_64_bounded_and_unbounded(gpu_engine):
    """64 live entries (the table's maximum): 32 bounded no-hit ranges of ragged sizes next to
    32 unbounded searches; exact exhaustion counts and valid winners."""
    roots = _roots(17, 64)
    counts = [1 + 977 * i for i in range(32)]
    bt = [gpu_engine.submit(r, M64, start=i << 40, device_mask=1, max_nonces_per_device=c)
          for i, (r, c) in enumerate(zip(roots[:32], counts))]
    ut = [gpu_engine.submit(r, LOW, device_mask=1) for r in roots[32:]]
    for c, t in zip(counts, bt):
        r = t.wait(60)
        assert r.status == _lib.NPOW_EXHAUSTED and r.nonces_done == c
    for root, t in zip(roots[32:], ut):
        r = t.wait(60)
        assert r.status == _lib.NPOW_OK and oracle.work_value(root, r.nonce) == r.value >= LOW


def test_new_job_does_not_wait_for_a_long_launch(gpu_engine):
    """With a 200-ms launch budget, a job submitted while another job's launch is running is
    searched within a few ms: the worker bumps the yield word, the running launch hands its
    unbounded job back (re-adopted with a new generation), and the next launch holds both."""
    gpu_engine.set_pool_tuning(budget_us=200_000)
    gpu_engine.reset_stats(0)
    try:
        tok = _lib.CancelToken()
        busy = gpu_engine.submit(bytes(range(32)), M64, device_mask=1, cancel=tok)
        time.sleep(0.05)  # the busy job's first 200-ms launch is running
        lat = []
        for r in _roots(18, 5):
            t0 = time.perf_counter()
            res = gpu_engine.submit(r, RECEIVE, device_mask=1).wait(10)
            lat.append(time.perf_counter() - t0)
            assert res.status == _lib.NPOW_OK and oracle.work_value(r, res.nonce) == res.value >= RECEIVE
        assert max(lat) < 0.1, lat
        assert busy.wait(0) is None  # still searching after being handed back
        tok.set()
        res = busy.wait(10)
        assert res.status == _lib.NPOW_CANCELLED and res.nonces_done > 0
    finally:
        gpu_engine.set_pool_tuning(budget_us=20_000)


def test_new_jobs_join_a_running_launch_and_finish_early(gpu_engine):
    """Two-group kernels, a launch of 2+ entries (counted): 8 receive-difficulty jobs submitted one
    after another beside two busy jobs in 200-ms launches each join the running launch as a dynamic
    entry (no yield) and return as soon as their entry's last workgroup has left it (early finish),
    not when the busy jobs' launch ends (its iteration cap, ~65 ms here); every count the kernel
    published equals the read-back after the launch, and all nonces add up to the device's counter."""
    gpu_engine.set_pool_tuning(budget_us=200_000)
    gpu_engine.reset_stats(0)
    try:
        toks = [_lib.CancelToken() for _ in range(2)]
        busy = [gpu_engine.submit(r, M64, device_mask=1, cancel=c) for r, c in zip(_roots(19, 2), toks)]
        time.sleep(0.05)  # their launch (2 entries: counted) is running
        lat, done = [], 0
        for r in _roots(18, 8):
            t0 = time.perf_counter()
            res = gpu_engine.submit(r, RECEIVE, device_mask=1).wait(10)
            lat.append(time.perf_counter() - t0)
            assert res.status == _lib.NPOW_OK and oracle.work_value(r, res.nonce) == res.value >= RECEIVE
            done += res.nonces_done
        assert max(lat) < 0.03 and sorted(lat)[len(lat) // 2] < 0.01, lat
        for c in toks:
            c.set()
        for t in busy:
            res = t.wait(10)
            assert res.status == _lib.NPOW_CANCELLED and res.nonces_done > 0
            done += res.nonces_done
        st = gpu_engine.stats(0)
        # (the busy pair's first launch held only the first of them: the second ended it, and a
        # receive job may have arrived before their two-entry launch started)
        assert st.dyn_entries >= len(lat) - 1 and st.yields <= 2, (st.dyn_entries, st.yields)
        assert st.early_finishes >= len(lat) and st.early_mismatches == 0, (st.early_finishes, st.early_mismatches)
        assert st.nonces == done
    finally:
        gpu_engine.set_pool_tuning(budget_us=20_000)


def test_launches_end_on_their_time_budget(gpu_engine):
    """A pool launch ends when its time budget is spent (every wave compares s_memrealtime with the
    launch's start, npow_kernel.hip pool_body_ls2), not at its iteration cap: a job that cannot win runs
    in launches of the budget's length (HIP-event kernel times, npow_device_stats), to within a few
    iterations of ~15 us."""
    budget_ms = 4.0
    gpu_engine.set_pool_tuning(budget_us=int(budget_ms * 1e3))
    try:
        tok = _lib.CancelToken()
        t = gpu_engine.submit(bytes(range(32)), M64, device_mask=1, cancel=tok)
        time.sleep(0.05)
        gpu_engine.reset_stats(0)
        time.sleep(0.3)
        st = gpu_engine.stats(0)
        tok.set()
        assert t.wait(10).status == _lib.NPOW_CANCELLED
        per = st.kernel_ms / max(1, st.launches)
        assert st.launches >= 40 and budget_ms - 0.1 <= per <= budget_ms + 0.25, (st.launches, st.kernel_ms)
    finally:
        gpu_engine.set_pool_tuning(budget_us=20_000)


def test_abandoned_ticket_is_cancelled_and_collected(gpu_engine):
    """A ticket dropped without wait() (a caller that gave up): its finaliser cancels the search
    and collects it, so the job leaves the pool and its cancel word is no longer read."""
    import gc
    tok = _lib.CancelToken()
    t = gpu_engine.submit(bytes(range(40, 72)), M64, device_mask=1, cancel=tok)
    assert t.wait(0.05) is None
    assert gpu_engine.pool_status()[1] >= 1
    del t, tok
    gc.collect()
    deadline = time.time() + 5
    while gpu_engine.pool_status() != (0, 0) and time.time() < deadline:
        time.sleep(0.01)
    assert gpu_engine.pool_status() == (0, 0)
    r = gpu_engine.submit(bytes(range(72, 104)), RECEIVE, device_mask=1).wait(30)  # the pool still serves
    assert r.status == _lib.NPOW_OK


def test_sweep_and_values_are_not_starved_by_endless_searches(gpu_engine):
    """Searches that never end keep the pool worker busy; a sweep and a values call still get
    the device (the worker drains its launches and hands it over) and the searches resume."""
    toks = [_lib.CancelToken() for _ in range(6)]
    ts = [gpu_engine.submit(r, M64, device_mask=1, cancel=c) for r, c in zip(_roots(19, 6), toks)]
    time.sleep(0.1)
    root = bytes(range(11, 43))
    t0 = time.perf_counter()
    hits = gpu_engine.sweep(root, 0xfff0000000000000, 0, 1 << 22, device_mask=1)
    vals = gpu_engine.values(root, 0, 4096)
    dt = time.perf_counter() - t0
    assert hits == oracle.sweep(root, 0xfff0000000000000, 0, 1 << 22)
    assert vals == oracle.work_values([root] * 4096, list(range(4096)))
    assert dt < 2.0, dt
    gpu_engine.reset_stats(0)
    time.sleep(0.1)
    assert gpu_engine.stats(0).launches > 0  # the searches are running again
    for c in toks:
        c.set()
    for t in ts:
        assert t.wait(30).status == _lib.NPOW_CANCELLED


def test_cpu_workers_beside_the_gpu():
    """--cpu-threads (nano-work-server.exe @1681064): 4 CPU worker threads as one more device of the pool,
    beside the GPU(s), in a process of its own (tests/cpu_workers_worker.py): CPU-only searches decided by
    the CPU device and re-validated by hashlib, exact bounded exhaustion, the first hit of a single-claim
    range, a hit only the CPU stride holds, GPU + CPU searches at receive difficulty, cancellation, and
    sweeps / values refused on the CPU device."""
    import json
    import os
    import subprocess
    import sys
    from conftest import ROOT
    p = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "cpu_workers_worker.py")],
                       capture_output=True, text=True, timeout=110)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-4000:]
    out = json.loads(p.stdout.strip().splitlines()[-1])
    print(json.dumps(out))
    assert out["ok"] and out["mixed_receive"]["cpu_nonces"] > 0


def test_wait_result_returns_at_the_decision(gpu_engine):
    """npow_wait_result (ABI 4): the outcome as soon as it is known -- a re-validated winner, a cancellation,
    an exhausted range -- with the ticket still valid for npow_wait, which then returns the same outcome and
    the complete nonce count."""
    eng = gpu_engine
    M64 = (1 << 64) - 1
    rng = random.Random(41)
    for _ in range(8):
        root = bytes(rng.getrandbits(8) for _ in range(32))
        t = eng.submit(root, 0xfffffe0000000000, start=rng.getrandbits(64), device_mask=1)
        r = t.wait_result(30)
        assert r.status == _lib.NPOW_OK and oracle.work_value_hashlib(root, r.nonce) == r.value >= 0xfffffe0000000000
        f = t.wait(30)
        assert f.status == _lib.NPOW_OK and (f.nonce, f.value) == (r.nonce, r.value) and f.nonces_done > 0
    tok = _lib.CancelToken()
    t = eng.submit(bytes(range(32)), M64, device_mask=1, cancel=tok)
    assert t.wait_result(0.2) is None
    tok.set()
    assert t.wait_result(10).status == _lib.NPOW_CANCELLED
    assert t.wait(10).status == _lib.NPOW_CANCELLED
    t = eng.submit(bytes(32), M64, start=5, device_mask=1, max_nonces_per_device=100_000)
    assert t.wait_result(30).status == _lib.NPOW_EXHAUSTED
    f = t.wait(30)
    assert f.status == _lib.NPOW_EXHAUSTED and f.nonces_done == 100_000


def test_a_long_search_does_not_spin_a_core(gpu_engine):
    """the win watcher spun one core for as long as any slot was armed (a whole long search, an idle
    lingering launch), and result waiters spun up to 50 ms per call.  Now both spin only within the job's spin window
    (~3x its expected time to a win, at most 50 ms -- the cap for a search that cannot end): over a second of an endless
    search nobody waits on, the process uses a fraction of a core (the pool worker's naps and the watcher's 20-us
    naps), not the one a spinning thread costs."""
    tok = _lib.CancelToken()
    t = gpu_engine.submit(bytes(range(100, 132)), M64, device_mask=1, cancel=tok)
    try:
        time.sleep(0.1)
        c0, w0 = time.process_time(), time.perf_counter()
        time.sleep(1.0)
        cores = (time.process_time() - c0) / (time.perf_counter() - w0)
    finally:
        tok.set()
    assert t.wait(10).status == _lib.NPOW_CANCELLED
    print({"process_cores_during_search": round(cores, 3)})
    assert cores < 0.75, cores

