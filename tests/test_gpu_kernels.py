"""Every search / sweep kernel variant the engine can select at npow_init, checked end to end
against the oracle in a child process (tests/kernel_variant_worker.py): the default two lockstep
workgroups per CU, one workgroup per CU (NANOPOW_LS_GROUPS=1) and the round-1 seq kernels
(NANOPOW_POOL_KERNEL=seq).  The rest of the GPU suite runs the default only."""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu

VARIANTS = {"ls2": {}, "ls1": {"NANOPOW_LS_GROUPS": "1"}, "seq": {"NANOPOW_POOL_KERNEL": "seq"}}


@pytest.mark.parametrize("variant", sorted(VARIANTS))
def test_kernel_variant(variant):
    env = dict(os.environ, **VARIANTS[variant])
    for k in ("NANOPOW_LS_GROUPS", "NANOPOW_POOL_KERNEL"):
        if k not in VARIANTS[variant]:
            env.pop(k, None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "kernel_variant_worker.py"), variant], env=env,
                       capture_output=True, text=True, timeout=110)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-4000:]
    out = json.loads(p.stdout.strip().splitlines()[-1])
    assert out["ok"] and out["variant"] == variant
