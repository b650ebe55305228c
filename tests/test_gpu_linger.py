"""Lingering launches (round 5, npow_kernel.hip ls2_linger; npow_pool.cpp Worker::end_linger): a search launch whose
entries are over waits in the GPU for the host's next dynamic entry, so a serial client's next root needs no launch.

Checked here: serial searches reuse launches (fewer launches than searches, the rest joined as dynamic entries) and
every result re-validates under hashlib; the nonce counts still add up to the device counter; a sweep, a values call
and a bounded search right after a search do not wait for the lingering launch's time budget (20 ms); the launch
ends on its own once idle; NANOPOW_LINGER=0 gives one launch per search; split searches over CU partitions.
Run on an MI355X: ``pytest -m gpu``.
"""
import json
import os
import random
import subprocess
import sys
import time

import pytest

import oracle
from conftest import ROOT
from nanopow import _lib

pytestmark = pytest.mark.gpu
RECEIVE, LOW = 0xfffffe0000000000, 0xfffff00000000000


def _roots(seed, n):
    rng = random.Random(seed)
    return [bytes(rng.getrandbits(8) for _ in range(32)) for _ in range(n)]


def _serial(eng, roots, thr, mask=1):
    done = 0
    for i, r in enumerate(roots):
        res = eng.submit(r, thr, start=i << 40, device_mask=mask).wait(30)
        assert res is not None and res.status == _lib.NPOW_OK, i
        assert oracle.work_value_hashlib(r, res.nonce) == res.value >= thr, i
        done += res.nonces_done
    return done


def test_serial_searches_join_the_lingering_launch(gpu_engine):
    time.sleep(0.05)  # an earlier test's lingering launch ends on its own (budget)
    gpu_engine.reset_stats(0)
    roots = _roots(51, 300)
    done = _serial(gpu_engine, roots, RECEIVE)
    st = gpu_engine.stats(0)
    # ~0.2 ms per search: a 20-ms launch serves its table entry and up to 32 dynamic entries
    assert st.launches < len(roots) // 4, (st.launches, st.dyn_entries)
    assert st.dyn_entries >= len(roots) // 2, (st.launches, st.dyn_entries)
    assert st.nonces == done
    assert st.early_mismatches == 0


def test_a_sweep_after_a_search_does_not_wait_for_the_budget(gpu_engine):
    root = _roots(52, 1)[0]
    gpu_engine.sweep(root, 0xffffffc000000000, 0, 1 << 22, device_mask=1)  # the first call loads the kernel (~20 ms)
    for trial in range(3):
        _serial(gpu_engine, _roots(53 + trial, 3), RECEIVE)
        t = time.perf_counter()
        hits = gpu_engine.sweep(root, 0xffffffc000000000, 0, 1 << 22, device_mask=1)
        dt = time.perf_counter() - t
        assert dt < 0.012, f"sweep took {dt * 1e3:.1f} ms behind a lingering launch"
        assert sorted(hits) == oracle.sweep(root, 0xffffffc000000000, 0, 1 << 22)


def test_values_and_bounded_searches_after_a_search(gpu_engine):
    root = _roots(54, 1)[0]
    gpu_engine.values(root, 0, 64, device=0)  # first calls load their kernels
    gpu_engine.submit(root, (1 << 64) - 1, start=0, device_mask=1, max_nonces_per_device=1 << 20).wait(30)
    for trial in range(3):
        _serial(gpu_engine, _roots(55 + trial, 3), RECEIVE)
        t = time.perf_counter()
        vals = gpu_engine.values(root, 1000, 4096, device=0)
        assert time.perf_counter() - t < 0.012
        assert vals == oracle.work_values([root] * 4096, [1000 + i for i in range(4096)])
        _serial(gpu_engine, _roots(58 + trial, 2), RECEIVE)
        t = time.perf_counter()
        res = gpu_engine.submit(root, (1 << 64) - 1, start=5 << 30, device_mask=1,
                                max_nonces_per_device=1 << 24).wait(30)
        dt = time.perf_counter() - t
        assert res.status == _lib.NPOW_EXHAUSTED and res.nonces_done == 1 << 24
        assert dt < 0.015, f"bounded search took {dt * 1e3:.1f} ms behind a lingering launch"


def test_an_idle_lingering_launch_ends(gpu_engine):
    """Idle past its time budget, the lingering launch ends (the worker raises end_linger, the kernel gives up after
    a budget's worth of waiting anyway): the next search starts a launch of its own instead of joining it."""
    _serial(gpu_engine, _roots(61, 2), RECEIVE)
    time.sleep(0.08)  # > the 20-ms budget
    assert gpu_engine.pool_status() == (0, 0)
    before = gpu_engine.stats(0)
    _serial(gpu_engine, _roots(62, 1), RECEIVE)
    after = gpu_engine.stats(0)
    assert after.launches == before.launches + 1 and after.dyn_entries == before.dyn_entries


def _child(env_extra, code):
    env = dict(os.environ, **env_extra)
    p = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=110,
                       cwd=ROOT)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-3000:]
    return json.loads(p.stdout.strip().splitlines()[-1])


CHILD = r"""
import json, random, sys
sys.path.insert(0, "nano-dpow_amd"); sys.path.insert(0, "oracle")
import nanopow, oracle
eng = nanopow.engine()
G = eng.n_devices
mask = (1 << G) - 1
rng = random.Random(71)
roots = [bytes(rng.getrandbits(8) for _ in range(32)) for _ in range(120)]
for d in range(G):
    eng.reset_stats(d)
done = 0
for i, r in enumerate(roots):
    res = eng.submit(r, 0xfffffe0000000000, start=i << 40, device_mask=mask).wait(30)
    assert res.status == 0 and oracle.work_value_hashlib(r, res.nonce) == res.value >= 0xfffffe0000000000, i
    done += res.nonces_done
st = [eng.stats(d) for d in range(G)]
print(json.dumps({"devices": G, "launches": sum(s.launches for s in st), "dyn": sum(s.dyn_entries for s in st),
                  "nonces": sum(s.nonces for s in st), "done": done,
                  "mismatch": sum(s.early_mismatches for s in st)}))
"""


def test_linger_off_gives_one_launch_per_search():
    out = _child({"NANOPOW_LINGER": "0"}, CHILD)
    assert out["dyn"] == 0 and out["launches"] >= 120
    assert out["nonces"] == out["done"] and out["mismatch"] == 0


def test_split_searches_linger_on_cu_partitions():
    out = _child({"NANOPOW_VIRTUAL_DEVICES": "4"}, CHILD)
    assert out["devices"] == 4
    assert out["launches"] < 4 * 120 // 4 and out["dyn"] >= 4 * 120 // 2, out
    assert out["nonces"] == out["done"] and out["mismatch"] == 0


def test_time_shared_devices_do_not_linger():
    """Logical devices time-sharing the whole GPU (NANOPOW_VIRTUAL_PARTITION=share): a lingering launch's sleeping
    waves would hold the CUs from the other devices' launches, so none lingers."""
    out = _child({"NANOPOW_VIRTUAL_DEVICES": "2", "NANOPOW_VIRTUAL_PARTITION": "share"}, CHILD)
    assert out["devices"] == 2 and out["dyn"] == 0
    assert out["nonces"] == out["done"] and out["mismatch"] == 0
