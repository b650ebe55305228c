"""Multi-device paths, in child processes (the engine's device set is fixed at npow_init).

On a one-GPU box the engine is opened with NANOPOW_VIRTUAL_DEVICES=G: G logical devices over the
physical GPU, each a partition of its CUs (a CU-masked stream over 256 / G CUs, the same number on every
XCD, npow_engine.cpp init_device; profiles/r04_cu_mask_probe.txt) with its own stream, buffers and pool
worker -- so every device's launch runs from its start on CUs of its own, as on separate GPUs.
NANOPOW_VIRTUAL_PARTITION=share makes them time-share the whole GPU instead (rounds 1-3).
* tests/multidev_worker.py (G = 4): the partitions (disjoint, equal), disjoint per-device strides, the
  winner from the right stride, exact per-device exhaustion, cancellation reaching every device,
  bursts and sweeps split over devices, subset masks.
* tests/sweep_split_worker.py (G = 2, 4, 8): BASELINE configs[2] at full size -- the 2^36 sweep of the
  fixture root split over G devices, bit-exact against tests/golden/sweep_2p36.json, the devices'
  nonce counters adding up to exactly 2^36.
* tests/overshoot_worker.py: first-found cancellation -- the nonces the losers' waves hashed after they knew
  (counted in the kernels, bounded exactly), the host-observed stop span against its mechanism (the kill's poll,
  one hash, the publish, the worker's look) and the launch budget, and no final count left unpublished -- on CU
  partitions (4 and 8 devices, and 4 with lingering launches forced on).
With two or more physical GPUs visible (and NANOPOW_VIRTUAL_DEVICES unset) the same workers also run
over the physical GPUs: the 2^36 sweep, the overshoot bound and a 64-root burst.  On a one-GPU box
those tests skip."""
import functools
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu

# First-found cancellation: what is asserted and what is recorded.
# * Hard, counted on the device: the losers' hashes after their waves knew (check_late).  Every losing workgroup but the
#   one whose poll read the kill word hashes exactly one more 512-lane hash, so a search is at most (G-1)(W-1)512.
# * The host-observed stop span (npow_wait_info.stop_after_decide_us) is bounded by its mechanism, not by one box's
#   percentile: the kill word is read by the next poll of a losing launch (one wave per iteration), the workgroups leave
#   after one more hash, the last one out publishes the final count, and the losing worker sees it at its next look (it
#   naps at most NAP_US between looks).  So MECHANISM_US = 2 iterations + NAP_US + PUBLISH_US, an iteration being one
#   hash of the device's whole grid at its measured kernel rate; the p50 must be within 2x of it.  The p99 must be far
#   below what a stop WITHOUT the kill path costs: the losing launch running on to its time budget (20 ms).  The
#   measured p50 / p99 / max are recorded (gpurun_out/latency_records.jsonl), not asserted.
# * No final count may go missing (npow_device_stats.stale_missing: a won or killed job of a lingering launch whose
#   count never came, though every launch that held it ended -- a protocol hole).  The worker's 1-ms fallback for a
#   count that is merely late (stale_drains, stale_late: the GPU published it late -- stale_gpu_delay_us, the publish
#   after the deciding win on the GPU's own clock) is recorded, not asserted: round 6 saw 8 such slots, all of one
#   search over 8 partitions, i.e. the whole GPU late at once, not a workgroup path that skips the publish.
NAP_US = 50.0       # npow_pool.cpp g_poll_us: a busy worker's longest nap between looks
PUBLISH_US = 20.0   # the final count's publish (32 loads, one pinned store) and the PCIe hop to the host
BUDGET_US = 20_000  # the launch's time budget: a loser the kill did not stop hashes until it ends
SEARCHES = "600"


def mechanism_us(out):
    """2 iterations of the slowest device's grid at its kernel rate + the worker's nap + the publish."""
    iter_us = max(out["iteration_us"])
    return 2.0 * iter_us + NAP_US + PUBLISH_US


def record(name, out):
    """Append the latency record for the round's evidence; no assertion depends on it."""
    d = os.path.join(ROOT, "gpurun_out")
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, "latency_records.jsonl"), "a") as f:
        f.write(json.dumps({"test": name, "stop_after_decide_us": out.get("stop_after_decide_us"),
                            "late_nonces_losers": out.get("late_nonces_losers"), "devices": out.get("devices"),
                            "mechanism_us": round(mechanism_us(out), 1) if "iteration_us" in out else None,
                            **{k: out.get(k) for k in ("stale_drains", "stale_late", "stale_missing",
                                                       "stale_gpu_delay_us", "linger_relays", "iteration_us")}})
                + "\n")


def check_stop_span(out):
    s = out["stop_after_decide_us"]
    mech = mechanism_us(out)
    assert s["p50"] < 2.0 * mech, (mech, out)
    assert s["p99"] < BUDGET_US / 4, out
    assert out["stale_missing"] == 0, out


def check_late(out, g):
    """The losers' hashes after they knew, counted in the kernels: each losing workgroup hashes at most one 512-lane hash
    after its waves knew (the dead word seen before a hash), the workgroups whose own poll read the kill word none -- so
    every search is at most (G-1)(W-1)512 for W workgroups per device, and a few polls more than one per device (two
    polls of a device reading the kill word before its relay lands) keep the median within 64 workgroups of it."""
    late, want = out["late_nonces_losers"], out["late_expected"]
    assert want == (g - 1) * (out["grid_per_device"] - 1) * 512, out
    assert out["late_max"] <= want and late["p50"] >= want - 64 * 512, out


def _child(script, env_extra, *args, timeout=110):
    """Run a worker with the engine's test hooks on: every HIP call site of every device checks that
    the calling thread's current HIP device is the device's own (npow_device_stats.affinity_checks); the worker
    reports the checks and failures, which must be > 0 and 0."""
    env = dict(os.environ, NANOPOW_TEST_HOOKS="1")
    for k, v in env_extra.items():
        if v is None:
            env.pop(k, None)
        else:
            env[k] = v
    p = subprocess.run([sys.executable, os.path.join(ROOT, "tests", script), *args], env=env,
                       capture_output=True, text=True, timeout=timeout)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-4000:]
    out = json.loads(p.stdout.strip().splitlines()[-1])
    print(json.dumps(out))
    checks, failures = out["affinity"]
    assert checks > 0 and failures == 0, out["affinity"]
    return out


@functools.lru_cache(maxsize=1)
def physical_gpus() -> int:
    """HIP devices the engine opens without NANOPOW_VIRTUAL_DEVICES (a child process: npow_init is
    process-wide)."""
    code = ("import sys; sys.path.insert(0, 'nano-dpow_amd'); from nanopow import _lib; "
            "print(_lib.Engine().n_devices)")
    env = {k: v for k, v in os.environ.items() if k != "NANOPOW_VIRTUAL_DEVICES"}
    p = subprocess.run([sys.executable, "-c", code], cwd=ROOT, env=env, capture_output=True, text=True, timeout=110)
    assert p.returncode == 0, p.stderr[-2000:]
    return int(p.stdout.strip().splitlines()[-1])


def _check_partitions(out, g):
    parts = out["partitions"]
    assert len(parts) == g
    if g > 1:
        assert all(first >= 0 for _hip, first, _cus in parts), parts  # CU partitions, not time-sharing


def test_four_logical_devices():
    out = _child("multidev_worker.py", {"NANOPOW_VIRTUAL_DEVICES": "4"})
    assert out["ok"] and out["devices"] == 4
    _check_partitions(out, 4)


@pytest.mark.parametrize("g", [2, 4, 8])
def test_sweep_2p36_split_over_devices(g):
    out = _child("sweep_split_worker.py", {"NANOPOW_VIRTUAL_DEVICES": str(g)})
    assert out["ok"] and out["devices"] == g and out["hits"] == 126
    assert sum(out["nonces_per_device"]) == 1 << 36
    _check_partitions(out, g)


@pytest.mark.parametrize("g,linger", [(4, None), (8, None), (4, "1")])
def test_first_win_overshoot_bound_cu_partitions(g, linger):
    """Lingering launches are on by default over 8 partitions (32 CUs each), off over 4; (4, "1") forces them on
    there too, where round 5 saw a won or killed entry's final count go unpublished (1 search in ~1,200)."""
    env = {"NANOPOW_VIRTUAL_DEVICES": str(g)}
    if linger is not None:
        env["NANOPOW_LINGER"] = linger
    out = _child("overshoot_worker.py", env, SEARCHES, "receive")
    assert out["ok"] and out["devices"] == g and out["kills_relayed"] > 0
    assert all(first >= 0 for _hip, first, _cus in out["partitions"]), out["partitions"]
    record(f"cu_partitions_{g}" + ("_linger" if linger else ""), out)
    check_late(out, g)
    check_stop_span(out)


def test_first_win_overshoot_time_shared_8_devices():
    """The rounds-1-3 rehearsal (8 logical devices time-sharing the whole GPU), kept for comparison: its
    tail is the time-sharing (a losing launch waits for CUs behind the other devices' launches)."""
    out = _child("overshoot_worker.py", {"NANOPOW_VIRTUAL_DEVICES": "8", "NANOPOW_VIRTUAL_PARTITION": "share"},
                 "200", "receive")
    assert out["ok"] and out["devices"] == 8 and out["kills_relayed"] > 0
    assert all(first < 0 for _hip, first, _cus in out["partitions"])
    record("time_shared_8", out)
    # time-sharing: a losing launch may wait for CUs behind the other devices' launches (up to one budget each); the
    # kill path, not the budget, must still stop the median search
    assert out["stop_after_decide_us"]["p50"] < BUDGET_US / 4, out


def _need_physical():
    if os.environ.get("NANOPOW_VIRTUAL_DEVICES"):
        pytest.skip("NANOPOW_VIRTUAL_DEVICES is set: the physical-GPU tests run without it")
    n = physical_gpus()
    if n < 2:
        pytest.skip(f"{n} physical GPU visible: the physical multi-GPU tests need 2 or more "
                    "(the CU-partition tests above stand in for them)")
    return n


def test_physical_gpus_sweep_2p36():
    n = _need_physical()
    out = _child("sweep_split_worker.py", {"NANOPOW_VIRTUAL_DEVICES": None, "EXPECT_DEVICES": str(n)})
    assert out["ok"] and out["devices"] == n and out["hits"] == 126
    assert sum(out["nonces_per_device"]) == 1 << 36
    assert len({hip for hip, _first, _cus in out["partitions"]}) == n  # one logical device per GPU


def test_physical_gpus_overshoot_bound():
    n = _need_physical()
    out = _child("overshoot_worker.py", {"NANOPOW_VIRTUAL_DEVICES": None}, "200", "receive")
    assert out["ok"] and out["devices"] == n and out["kills_relayed"] > 0
    record(f"physical_{n}", out)
    check_late(out, n)
    check_stop_span(out)


def test_physical_gpus_burst_64():
    n = _need_physical()
    out = _child("multidev_worker.py", {"NANOPOW_VIRTUAL_DEVICES": None, "EXPECT_DEVICES": str(n)}, "burst")
    assert out["ok"] and out["devices"] == n
