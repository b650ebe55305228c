"""Shared test setup.

* ``gpu`` marker: tests that need an MI355X (run with ``-m gpu`` on the GPU box).
* Paths: the product package lives in ``nano-dpow_amd/`` (``import nanopow``);
  the parity checker in ``oracle/`` (test infrastructure only).
* GPU tests build nothing: they load the in-tree ``libnanopow.so`` and fail
  loudly if it (or the GPU) is missing -- there is no CPU fallback to pass on.
"""
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "nano-dpow_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X GPU (libnanopow HIP path)")


# Run order of the GPU suite: under `pytest -x` the first failure hides every test after it, and
# collection is alphabetical by file.  So the bit-exact parity tests and the JSON drop-in go first, then the pool,
# sanitizers, faults and the BASELINE configs, and the tests whose subject is latency (stop spans, lingering
# launches) last.  Files not named here keep their place after the named ones, in collection order.
GPU_ORDER = ["test_gpu_parity.py", "test_gpu_server.py", "test_gpu_kernels.py", "test_gpu_pool.py",
             "test_gpu_sanitizers.py", "test_gpu_faults.py", "test_gpu_exit.py", "test_gpu_configs.py",
             "test_gpu_linger.py", "test_gpu_multidevice.py"]
# ... and within a file these go after the rest of it
LATENCY_LAST = ("test_first_win_overshoot",)


def _order_key(item):
    fname = os.path.basename(str(item.fspath))
    rank = GPU_ORDER.index(fname) if fname in GPU_ORDER else len(GPU_ORDER)
    latency = any(item.name.startswith(p) for p in LATENCY_LAST)
    return (1 if latency else 0, rank)


def pytest_collection_modifyitems(session, config, items):
    # a stable sort: the order within each (latency, file) group is the collection order
    items[:] = sorted(items, key=_order_key)


def load_golden(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def golden():
    return load_golden


@pytest.fixture(scope="session")
def gpu_engine():
    import nanopow
    eng = nanopow.engine()  # raises NanoPowError if libnanopow.so or the GPU is missing
    assert eng.n_devices >= 1
    return eng
