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
