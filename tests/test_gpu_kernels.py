"""The search / sweep kernels end to end in a fresh process (tests/kernel_variant_worker.py): first-win
searches, one launch table with several entries, bounded exhaustion after exactly its nonce budget, a
bounded hit at the very end of its range, an exhaustive sweep against the oracle.  Since round 3 the
engine ships one kernel shape (npow_pool_kernel_ls2*, npow_sweep_kernel_ls2: two lockstep workgroups
per CU); the round-2 alternatives (one workgroup per CU, the seq kernels) were removed with their
NANOPOW_LS_GROUPS / NANOPOW_POOL_KERNEL switches."""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


def test_shipped_kernels_end_to_end():
    env = dict(os.environ)
    for k in ("NANOPOW_LS_GROUPS", "NANOPOW_POOL_KERNEL"):  # removed switches: must change nothing
        env[k] = "1" if k == "NANOPOW_LS_GROUPS" else "seq"
    p = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "kernel_variant_worker.py"), "ls2"], env=env,
                       capture_output=True, text=True, timeout=110)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-4000:]
    out = json.loads(p.stdout.strip().splitlines()[-1])
    assert out["ok"] and out["variant"] == "ls2" and out["pool_groups"] == 4
