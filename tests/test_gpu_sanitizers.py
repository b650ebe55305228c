"""Host-sanitizer runs of the C ABI on the GPU (DESIGN.md "Host sanitizers").

tools/abi_asan_driver and tools/abi_tsan_driver are the engine, pool and kernel sources
built with -fsanitize=address / thread on the host side (``make -C nano-dpow_amd/csrc asan
tsan``, run by ``__graft_entry__.build()``); each drives every entry point from several
threads and checks every GPU result against the library's CPU value.  A sanitizer report
makes the driver exit non-zero (halt_on_error).
"""
import os
import subprocess

import pytest

from conftest import ROOT

TOOLS = os.path.join(ROOT, "tools")


def _run(binary, env_extra):
    path = os.path.join(TOOLS, binary)
    assert os.path.exists(path), f"{binary} not built: run __graft_entry__.build()"
    env = dict(os.environ, **env_extra)
    out = subprocess.run([path], capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    log = out.stdout + out.stderr
    assert out.returncode == 0, log[-4000:]
    assert "abi_asan_driver: ok (0 failures)" in log, log[-4000:]
    assert "Sanitizer" not in log.replace("Suppressions used", ""), log[-4000:]


@pytest.mark.gpu
def test_c_abi_under_address_sanitizer():
    _run("abi_asan_driver", {"ASAN_OPTIONS": "detect_leaks=1:halt_on_error=1",
                             "LSAN_OPTIONS": "suppressions=tools/lsan.supp"})


@pytest.mark.gpu
def test_c_abi_under_thread_sanitizer():
    _run("abi_tsan_driver", {"TSAN_OPTIONS": "suppressions=tools/tsan.supp:halt_on_error=1"})


@pytest.mark.gpu
def test_smoke_under_undefined_behaviour_sanitizer():
    """__graft_entry__.smoke() through libnanopow_ubsan.so (host-side -fsanitize=undefined)."""
    lib = os.path.join(ROOT, "nano-dpow_amd", "nanopow", "libnanopow_ubsan.so")
    assert os.path.exists(lib), "libnanopow_ubsan.so not built: run __graft_entry__.build()"
    code = ("import __graft_entry__ as g; g.smoke(); "
            "print('loaded', open('/proc/self/maps').read().count('libnanopow_ubsan.so') > 0)")
    env = dict(os.environ, NANOPOW_LIB=lib, UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    out = subprocess.run(["python", "-c", code], capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    log = out.stdout + out.stderr
    assert out.returncode == 0, log[-4000:]
    assert "loaded True" in out.stdout and "runtime error" not in log, log[-4000:]
