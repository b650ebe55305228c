"""Multi-device first-win on a one-GPU box: the engine opened with NANOPOW_VIRTUAL_DEVICES=4
(four logical devices over the physical GPU, each with its own stream, buffers and pool
worker) in a child process -- disjoint per-device strides, the winner from the right stride,
exact per-device exhaustion, cancellation reaching every device, bursts and sweeps split over
devices, subset masks (tests/multidev_worker.py)."""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


def test_four_logical_devices():
    env = dict(os.environ, NANOPOW_VIRTUAL_DEVICES="4")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "multidev_worker.py")], env=env,
                       capture_output=True, text=True, timeout=110)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-4000:]
    out = json.loads(p.stdout.strip().splitlines()[-1])
    assert out["ok"] and out["devices"] == 4
