"""GPU parity: the HIP path (through the C ABI) against the oracle and the golden fixtures.

Bit-exact throughout (integer work).  Run on an MI355X: ``pytest -m gpu``.
Covers: every golden (root, nonce, value) triple through all three GPU hash paths
(npow_values = the stream the search and sweep kernels run, the seq stream, the generic
per-lane-root kernel); contiguous value ranges incl. 2^32 and 2^64 carries and 2^20 / 2^24
ranges, 2^28 consecutive values of the shipped stream for two roots and 2^32 for a third; every exhaustive sweep
fixture (8 roots x [0, 2^28), hashlib ranges, the range across 2^64 -> 0) and,
at BASELINE config 3's full size, the 2^36 sweep; first-win search validity
at the BASELINE thresholds; threshold edges; exhaustion, cancellation,
empty / ragged ranges; multi-device masks.
"""
import os
import random
import threading
import time

import numpy as np
import pytest

import oracle
from conftest import load_golden
from nanopow import _lib

pytestmark = pytest.mark.gpu
M64 = (1 << 64) - 1
SEND, RECEIVE, LOW = 0xfffffff800000000, 0xfffffe0000000000, 0xfffff00000000000


def test_native_library_is_the_hip_path(gpu_engine):
    assert "gfx950" in gpu_engine.version()
    assert gpu_engine.abi_version() == _lib.NPOW_ABI_VERSION
    st = gpu_engine.stats(0)
    assert st.cus >= 1 and st.grid == 4 * st.cus and st.pool_groups == 4


def bench_root(i: int) -> bytes:
    """bench.py's roots R_i = blake2b(b"nanopow-bench" + LE64(i), 32)."""
    import hashlib
    return hashlib.blake2b(b"nanopow-bench" + i.to_bytes(8, "little"), digest_size=32).digest()


def test_config1_send_difficulty_serial_on_one_gpu(gpu_engine):
    """BASELINE configs[1] as bench.py runs it: one MI355X, one block hash at a time at the send
    difficulty fffffff800000000, each search submitted, its result taken at the decision (npow_wait_result, what a
    work_generate reply carries) and the ticket collected (npow_wait).  Every winner re-validates under hashlib (the
    reference CPU path), and the sample's nonce counts follow the exponential law of a first hit at p = 2^-29 (a
    Kolmogorov-Smirnov test against Exp(2^29); the few hundred thousand nonces a launch hashes after its win are 0.1 %
    of the mean).  Times are recorded, not asserted."""
    from scipy import stats
    n = 128
    done, ttw = [], []
    for i in range(n):
        root = bench_root(10_000 + i)
        t0 = time.perf_counter()
        t = gpu_engine.submit(root, SEND, start=0, device_mask=1)
        r = t.wait_result(60)
        ttw.append(time.perf_counter() - t0)
        assert r is not None and r.status == _lib.NPOW_OK, i
        assert oracle.work_value_hashlib(root, r.nonce) == r.value >= SEND, i
        f = t.wait(60)
        assert (f.status, f.nonce, f.value) == (r.status, r.nonce, r.value) and f.nonces_done > 0
        done.append(f.nonces_done)
    mean = float(1 << 29)
    ks = stats.kstest(np.array(done, dtype=np.float64), "expon", args=(0, mean))
    assert ks.pvalue > 1e-3, (ks, np.mean(done) / mean)
    # the mean within 4.5 standard errors (an exponential's sd is its mean)
    assert abs(np.mean(done) / mean - 1.0) < 4.5 / np.sqrt(n), np.mean(done) / mean
    rec = {"test": "config1_send_serial", "searches": n, "ks_pvalue": round(float(ks.pvalue), 4),
           "mean_nonces_over_2p29": round(float(np.mean(done)) / mean, 4),
           "ttw_ms_p50": round(float(np.median(ttw)) * 1e3, 3), "ttw_ms_p99": round(float(np.percentile(ttw, 99)) * 1e3, 3)}
    d = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out")
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, "latency_records.jsonl"), "a") as fh:
        import json
        fh.write(json.dumps(rec) + "\n")


PATHS = pytest.mark.parametrize("path", [_lib.NPOW_PATH_SEARCH, _lib.NPOW_PATH_SEQ], ids=["search_stream", "seq_stream"])


@PATHS
def test_golden_triples(gpu_engine, path):
    """Every golden (root, nonce, value) triple (hashlib) through one hash path, one root at a time:
    NPOW_PATH_SEARCH is the instruction stream the search and sweep kernels execute
    (npow_values_kernel_ls2 -- the same uniform loads, priority runs and four 512-lane
    workgroups per CU), so its full 64-bit values are compared, not only its hit decisions."""
    g = load_golden("work_values.json")["triples"]
    got = [gpu_engine.values(bytes.fromhex(r), int(n, 16), 1, path=path)[0] for r, n, _ in g]
    assert [f"{v:016x}" for v in got] == [v for _, _, v in g]


def test_golden_triples_generic_path(gpu_engine):
    """The same triples through the per-lane-root kernel (npow_values_pairs), in one launch."""
    g = load_golden("work_values.json")["triples"]
    roots = [bytes.fromhex(r) for r, _, _ in g]
    nonces = [int(n, 16) for _, n, _ in g]
    assert gpu_engine.values_pairs(roots, nonces) == [int(v, 16) for _, _, v in g]


@PATHS
@pytest.mark.parametrize("start,count", [
    (0, 1 << 16), (0xffffffff - 1000, 5000), ((1 << 64) - 3000, 6000), (12345, 1), (7, 65), (99, 64 * 1000 + 17),
    ((1 << 32) - (1 << 19), 1 << 20), (0x0123456789abcdef, 1 << 20), ((1 << 64) - (1 << 19) - 3, 1 << 20)])
def test_value_ranges_vs_oracle(gpu_engine, path, start, count):
    """Contiguous ranges: ragged lengths (1, 65, 64k+17: partial rows and blocks), the 2^32 carry
    into the nonce's high word and the 2^64 wrap, and 2^20-nonce ranges across both."""
    rng = random.Random(start ^ count)
    root = bytes(rng.getrandbits(8) for _ in range(32))
    got = gpu_engine.values_array(root, start, count, path=path)
    want = oracle.work_values_range(root, start, count)
    assert got.tolist() == want.tolist()


def test_value_range_2p24_both_streams(gpu_engine):
    """2^24 consecutive values (one full values launch) through both generated streams, equal to
    each other and to the oracle's on every nonce."""
    root = bytes.fromhex("E89208DD038FBB269987689621D52292AE9C35941A7484756ECCED92A65093BA")
    start = 0x62f05417dd3fb691 - (1 << 23)
    a = gpu_engine.values_array(root, start, 1 << 24, path=_lib.NPOW_PATH_SEARCH)
    b = gpu_engine.values_array(root, start, 1 << 24, path=_lib.NPOW_PATH_SEQ)
    want = oracle.work_values_range(root, start, 1 << 24)
    assert (a == want).all() and (b == want).all()
    assert int(a[1 << 23]) == 0xfffffff4000d3dac  # the Nano genesis work


def test_value_range_2p28_shipped_stream(gpu_engine):
    """2^28 consecutive full 64-bit values of the stream the search and sweep kernels execute, every
    one equal to the oracle's: 16 launches of 2^24 across the 2^40 carry of the nonce (bit 40 set
    mid-range), for two roots.  The oracle side runs on the box's CPUs (~3 s per root)."""
    for root_hex, start in (("7A0C6E2F1B3D5948E6A1C2B3D4E5F60718293A4B5C6D7E8F90A1B2C3D4E5F607", (1 << 40) - (1 << 27)),
                            ("E89208DD038FBB269987689621D52292AE9C35941A7484756ECCED92A65093BA", 0x62f05417dd3fb691)):
        root = bytes.fromhex(root_hex)
        for k in range(16):
            s = (start + (k << 24)) & ((1 << 64) - 1)
            got = gpu_engine.values_array(root, s, 1 << 24, path=_lib.NPOW_PATH_SEARCH)
            want = oracle.work_values_range(root, s, 1 << 24)
            bad = np.flatnonzero(got != want)
            assert bad.size == 0, f"root {root_hex[:8]}: {bad.size} values differ from {s + int(bad[0]):#x} on"


def test_value_range_2p32_shipped_stream(gpu_engine):
    """2^32 consecutive full 64-bit values of the shipped stream -- a whole 32-bit nonce span, across the carry into bit
    32 -- every one equal to the oracle's (north_star: "identical 64-bit work values for any nonce"): 256 launches of
    2^24, each compared in full with the C oracle on the box's CPUs (16 threads).  Also a checksum: the values' sum
    mod 2^64 over the whole span, GPU against oracle."""
    root = bytes.fromhex("3B7F1E0C9A2D4F6B8C1E3A5D7F9B0C2E4A6D8F1B3C5E7A9D0F2B4C6E8A1D3F5B")
    start = (1 << 31) * 3  # [3 * 2^31, 5 * 2^31): bit 32 carries at 2^32 (a quarter in) and bit 33 at 2^33
    total_gpu = total_cpu = 0
    for k in range(256):
        s = start + (k << 24)
        got = gpu_engine.values_array(root, s, 1 << 24, path=_lib.NPOW_PATH_SEARCH)
        want = oracle.work_values_range(root, s, 1 << 24)
        bad = np.flatnonzero(got != want)
        assert bad.size == 0, f"{bad.size} values differ from {s + int(bad[0]):#x} on"
        total_gpu = (total_gpu + int(got.sum(dtype=np.uint64))) & ((1 << 64) - 1)
        total_cpu = (total_cpu + int(want.sum(dtype=np.uint64))) & ((1 << 64) - 1)
    assert total_gpu == total_cpu


def test_sweep_fixtures(gpu_engine):
    for c in load_golden("sweeps_small.json")["cases"]:
        got = gpu_engine.sweep(bytes.fromhex(c["root"]), int(c["threshold"], 16), int(c["start"], 16), c["count"])
        assert [f"{h:016x}" for h in got] == c["hits"], c["method"]


def test_sweep_2p30_hashlib_fixture(gpu_engine):
    """[0, 2^30) of the config-3 root at fffff000: ~1,024 hits, fixture from hashlib alone."""
    g = load_golden("sweep_2p30_hashlib.json")
    got = gpu_engine.sweep(bytes.fromhex(g["root"]), int(g["threshold"], 16), 0, g["count"], cap=1 << 12)
    assert [f"{h:016x}" for h in got] == g["hits"]


def test_sweep_2p36_full_size(gpu_engine):
    """BASELINE config 3: exhaustive 2^36 sweep, bit-exact hit set vs the CPU fixture."""
    path = os.path.join(os.path.dirname(__file__), "golden", "sweep_2p36.json")
    if not os.path.exists(path):
        pytest.skip("sweep_2p36.json not generated")
    g = load_golden("sweep_2p36.json")
    t = time.time()
    got = gpu_engine.sweep(bytes.fromhex(g["root"]), int(g["threshold"], 16), 0, g["count"], cap=1 << 12)
    dt = time.time() - t
    assert [f"{h:016x}" for h in got] == g["hits"]
    print(f"2^36 sweep: {len(got)} hits in {dt:.2f} s = {(1 << 36) / dt / 1e9:.2f} Gnonce/s")


def test_sweep_ragged_multi_launch_subranges(gpu_engine):
    """Sweep launches claim 64-nonce runs from a counter that alternates between two cache
    lines by launch parity: ragged sub-ranges of the 2^36 fixture spanning 1-3 launches
    (2^31 nonces each) return exactly the fixture's hits inside them."""
    g = load_golden("sweep_2p36.json")
    root, thr = bytes.fromhex(g["root"]), int(g["threshold"], 16)
    hits = [int(h, 16) for h in g["hits"]]
    for lo, n in [(12345, (1 << 31) + 77), (5 << 33, (3 << 31) - 1), (hits[3] - 1, 2)]:
        want = [h for h in hits if lo <= h < lo + n]
        assert gpu_engine.sweep(root, thr, lo, n, cap=1 << 12) == want, (lo, n)


def test_sweep_every_nonce_a_hit_exactly_once(gpu_engine):
    """Threshold 0 makes every nonce a hit: the claim counter covers each nonce exactly once,
    also for a count that is not a multiple of 64 or of the claim size (one launch; the
    device hit buffer holds 2^20)."""
    root = bytes(range(5, 37))
    n = 1_000_003
    got = gpu_engine.sweep(root, 0, 1 << 50, n, cap=n)
    assert got == [(1 << 50) + i for i in range(n)]


def test_sweep_edges(gpu_engine):
    root = bytes(range(32))
    assert gpu_engine.sweep(root, 0, 5, 0) == []
    # threshold 0: every nonce is a hit (exact count, order, ragged length)
    got = gpu_engine.sweep(root, 0, 100, 1000, cap=2000)
    assert got == list(range(100, 1100))
    got = gpu_engine.sweep(root, 0, M64 - 9, 20, cap=100)  # wraps 2^64 -> 0
    assert got == [(M64 - 9 + i) & M64 for i in range(20)]
    # threshold = an exact value: the nonce with that value is a hit (>=), value+1 excludes it
    vals = gpu_engine.values(root, 0, 4096)
    top = max(range(4096), key=lambda i: vals[i])
    assert gpu_engine.sweep(root, vals[top], 0, 4096) == [top]
    assert gpu_engine.sweep(root, vals[top] + 1, 0, 4096) == []


def test_sweep_capacity_error(gpu_engine):
    with pytest.raises(_lib.NanoPowError) as ei:
        gpu_engine.sweep(bytes(32), 0, 0, 5000, cap=100)
    assert ei.value.code == _lib.NPOW_ERR_CAPACITY


@pytest.mark.parametrize("thr", [LOW, RECEIVE, SEND])
def test_search_results_revalidate(gpu_engine, thr):
    rng = random.Random(thr)
    n = 64
    done = 0
    for _ in range(n):
        root = bytes(rng.getrandbits(8) for _ in range(32))
        r = gpu_engine.search(root, thr, start=rng.getrandbits(64))
        assert r.status == _lib.NPOW_OK
        assert oracle.work_value_hashlib(root, r.nonce) == r.value >= thr
        assert r.nonces_done > 0
        done += r.nonces_done
    # nonces per search: a geometric number with mean 2^64 / (2^64 - thr) plus the rest of the
    # launch after the win; over 64 searches the mean stays within a factor 3 of the expectation
    expect = (1 << 64) / ((1 << 64) - thr)
    assert expect / 3 < done / n < 3 * expect + (1 << 22), (done / n, expect)


def test_search_is_first_in_small_ranges(gpu_engine):
    """With one launch covering [start, start+count) the winner must be a real hit of that
    range (any of them: lanes race), and exhaustion must be reported when there is none."""
    c = load_golden("sweeps_small.json")["cases"][1]  # RECEIVE hits of root 0 in [0, 2^28)
    root, thr = bytes.fromhex(c["root"]), int(c["threshold"], 16)
    hits = [int(h, 16) for h in c["hits"]]
    r = gpu_engine.search(root, thr, start=0, max_nonces_per_device=1 << 28)
    assert r.status == _lib.NPOW_OK and r.nonce in hits
    # a range with no hit: between two consecutive hits
    a, b = hits[0], hits[1]
    r = gpu_engine.search(root, thr, start=a + 1, max_nonces_per_device=b - a - 1)
    assert r.status == _lib.NPOW_EXHAUSTED and r.nonce is None
    assert r.nonces_done == b - a - 1


def test_search_threshold_edges(gpu_engine):
    root = bytes(32)
    r = gpu_engine.search(root, 0, start=42)
    assert r.status == _lib.NPOW_OK and r.value == oracle.work_value(root, r.nonce)
    r = gpu_engine.search(root, M64, start=0, max_nonces_per_device=1 << 22)
    assert r.status == _lib.NPOW_EXHAUSTED


def test_search_cancel_from_another_thread(gpu_engine):
    tok = _lib.CancelToken()
    out = {}
    th = threading.Thread(target=lambda: out.setdefault("r", gpu_engine.search(bytes(32), M64, cancel=tok)))
    t0 = time.time()
    th.start()
    time.sleep(0.2)
    tok.set()
    th.join(10)
    assert not th.is_alive()
    assert out["r"].status == _lib.NPOW_CANCELLED
    assert out["r"].nonces_done > 0
    assert time.time() - t0 < 5


def test_blocking_search_releases_the_gil(gpu_engine):
    """npow_search blocks its caller's thread inside the library with the GIL released
    (ctypes.CDLL): Python code in other threads keeps running at full speed meanwhile."""
    def spin(seconds):
        n, end = 0, time.perf_counter() + seconds
        while time.perf_counter() < end:
            n += 1
        return n
    alone = spin(0.2)
    tok = _lib.CancelToken()
    th = threading.Thread(target=lambda: gpu_engine.search(bytes(range(9, 41)), M64, cancel=tok))
    th.start()
    time.sleep(0.05)
    beside = spin(0.2)
    tok.set()
    th.join(10)
    assert not th.is_alive()
    assert beside > 0.5 * alone, (beside, alone)


def test_device_masks(gpu_engine):
    root = bytes(range(1, 33))
    n = gpu_engine.n_devices
    r = gpu_engine.search(root, RECEIVE, device_mask=(1 << n) - 1)
    assert r.status == _lib.NPOW_OK and oracle.work_value(root, r.nonce) >= RECEIVE
    with pytest.raises(_lib.NanoPowError):
        gpu_engine.search(root, RECEIVE, device_mask=1 << 40)


def test_search_batch(gpu_engine):
    rng = random.Random(5)
    roots = [bytes(rng.getrandbits(8) for _ in range(32)) for _ in range(16)]
    thr = [RECEIVE] * 15 + [M64]
    toks = [None] * 15 + [_lib.CancelToken()]
    toks[15].set()
    res, done = gpu_engine.search_batch(roots, thr, cancels=toks)
    for root, r in zip(roots[:15], res[:15]):
        assert r.status == _lib.NPOW_OK and oracle.work_value(root, r.nonce) == r.value >= RECEIVE
    assert res[15].status == _lib.NPOW_CANCELLED
    assert done > 0


def test_stats_count_every_nonce(gpu_engine):
    gpu_engine.reset_stats(0)
    gpu_engine.sweep(bytes(32), SEND, 0, 10_000_019)
    st = gpu_engine.stats(0)
    assert st.nonces == 10_000_019 and st.launches >= 1 and st.kernel_ms > 0


def test_abi2_stats_call_writes_only_its_prefix(gpu_engine):
    """npow_device_stats_get (the ABI-2 call) writes the struct only up to dyn_entries, as a caller
    compiled against the round-2 header allocates it; npow_device_stats_get_sized writes what it is
    told (the struct grew while the call kept its signature)."""
    import ctypes
    lib = gpu_engine.lib
    buf = (ctypes.c_uint8 * ctypes.sizeof(_lib.DeviceStats))(*([0xA5] * ctypes.sizeof(_lib.DeviceStats)))
    prefix = _lib.DeviceStats.kills_relayed.offset
    assert lib.npow_device_stats_get(0, ctypes.cast(buf, ctypes.POINTER(_lib.DeviceStats))) == 0
    assert bytes(buf[prefix:]) == b"\xa5" * (len(buf) - prefix)
    assert lib.npow_device_stats_get_sized(0, ctypes.cast(buf, ctypes.POINTER(_lib.DeviceStats)), 16) == 0
    assert bytes(buf[prefix:]) == b"\xa5" * (len(buf) - prefix)
    st = gpu_engine.stats(0)
    assert st.pool_groups == 4 and st.cus > 0


def test_wait_info_single_device(gpu_engine):
    """npow_wait_info on a one-device search: the winner is that device, the decision precedes the
    finish, no other device to overshoot; the result re-validates under hashlib."""
    root = bytes(range(100, 132))
    info = gpu_engine.submit(root, RECEIVE, start=77, device_mask=1).wait_info(30)
    assert info.status == _lib.NPOW_OK and info.winner_device == 0 and info.n_devices == 1
    assert 0 < info.decide_us <= info.finish_us
    assert info.stop_after_decide_us == 0 and info.overshoot_nonces == 0
    assert oracle.work_value_hashlib(root, info.nonce) == info.value >= RECEIVE
    assert info.nonces_done > 0
