"""GPU fault policy (SURVEY.md §5 failure recovery; nano-work-server.exe @1669040 / @1669144):
a device that returns invalid work 3 times in a row, or whose HIP calls fail, is dropped, and
the jobs it held are re-strided onto the surviving devices.  Each scenario runs in a child
process with NANOPOW_VIRTUAL_DEVICES (logical devices over the one physical GPU) and one of the
engine's fault-injection hooks (tests/fault_worker.py)."""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu

SCENARIOS = {
    "invalid": {"NANOPOW_VIRTUAL_DEVICES": "8", "NANOPOW_FAULT_INVALID": "3", "NANOPOW_TEST_HOOKS": "1"},
    "hip": {"NANOPOW_VIRTUAL_DEVICES": "8", "NANOPOW_FAULT_HIP": "2:3", "NANOPOW_TEST_HOOKS": "1"},
    "exhaust": {"NANOPOW_VIRTUAL_DEVICES": "8", "NANOPOW_FAULT_HIP": "2:3", "NANOPOW_TEST_HOOKS": "1"},
    "allbad": {"NANOPOW_VIRTUAL_DEVICES": "2", "NANOPOW_FAULT_INVALID": "0,1", "NANOPOW_TEST_HOOKS": "1"},
    "init": {"NANOPOW_VIRTUAL_DEVICES": "4", "NANOPOW_FAULT_INIT": "2", "NANOPOW_TEST_HOOKS": "1"},
    "hooks_off": {"NANOPOW_VIRTUAL_DEVICES": "2", "NANOPOW_FAULT_INVALID": "0,1", "NANOPOW_FAULT_INIT": "0"},
    "cpu_last": {"NANOPOW_VIRTUAL_DEVICES": "1", "NANOPOW_FAULT_HIP": "0:0", "NANOPOW_TEST_HOOKS": "1",
                 "NANOPOW_TEST_CPU_RELEASE_DELAY_US": "1500000"},
    "affinity": {"NANOPOW_VIRTUAL_DEVICES": "2", "NANOPOW_TEST_AFFINITY_SKEW": "1", "NANOPOW_TEST_HOOKS": "1"},
}


@pytest.mark.parametrize("scenario", sorted(SCENARIOS))
def test_fault_scenario(scenario):
    env = dict(os.environ, **SCENARIOS[scenario])
    if "NANOPOW_TEST_HOOKS" not in SCENARIOS[scenario]:
        env.pop("NANOPOW_TEST_HOOKS", None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "fault_worker.py"), scenario], env=env,
                       capture_output=True, text=True, timeout=110)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-4000:]
    out = json.loads(p.stdout.strip().splitlines()[-1])
    assert out["ok"] and out["scenario"] == scenario
    if scenario == "hooks_off":
        assert "ignored" in p.stderr and "TEST HOOKS ACTIVE" not in p.stderr
