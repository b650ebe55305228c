"""Multi-device paths on a one-GPU box: the engine opened with NANOPOW_VIRTUAL_DEVICES=G (G logical
devices over the physical GPU, each with its own stream, buffers and pool worker) in a child
process.
* tests/multidev_worker.py (G = 4): disjoint per-device strides, the winner from the right stride,
  exact per-device exhaustion, cancellation reaching every device, bursts and sweeps split over
  devices, subset masks.
* tests/sweep_split_worker.py (G = 2, 4, 8): BASELINE configs[2] at full size -- the 2^36 sweep of
  the fixture root split over G devices, bit-exact against tests/golden/sweep_2p36.json, the devices'
  nonce counters adding up to exactly 2^36.
* tests/overshoot_worker.py (G = 8): first-found cancellation -- after the host accepts a winner the
  other devices stop within a bounded time (median under 0.5 ms, host-observed)."""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


def _child(script, env_extra, *args, timeout=110):
    env = dict(os.environ, **env_extra)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "tests", script), *args], env=env,
                       capture_output=True, text=True, timeout=timeout)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-4000:]
    out = json.loads(p.stdout.strip().splitlines()[-1])
    print(json.dumps(out))
    return out


def test_four_logical_devices():
    out = _child("multidev_worker.py", {"NANOPOW_VIRTUAL_DEVICES": "4"})
    assert out["ok"] and out["devices"] == 4


@pytest.mark.parametrize("g", [2, 4, 8])
def test_sweep_2p36_split_over_devices(g):
    out = _child("sweep_split_worker.py", {"NANOPOW_VIRTUAL_DEVICES": str(g)})
    assert out["ok"] and out["devices"] == g and out["hits"] == 126
    assert sum(out["nonces_per_device"]) == 1 << 36


def test_first_win_overshoot_bound_8_devices():
    out = _child("overshoot_worker.py", {"NANOPOW_VIRTUAL_DEVICES": "8"}, "200", "receive")
    assert out["ok"] and out["devices"] == 8 and out["kills_relayed"] > 0
    assert out["stop_after_decide_us"]["p50"] < 500.0, out
