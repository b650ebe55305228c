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
    _run("abi_asan_driver", {"ASAN_OPTIONS": "detect_leaks=1:halt_on_error=1:verify_asan_link_order=0",
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


@pytest.mark.gpu
@pytest.mark.parametrize("binary", ["abi_asan_driver", "abi_tsan_driver"])
def test_device_drop_under_sanitizers(binary):
    """The fault policy's paths (a device dropped after 3 invalid results, its jobs re-strided onto
    the others) under ASan / TSan: 4 logical devices, device 1's wins corrupted, every search,
    ticket and bounded range over all devices (DRIVER_MASK=0)."""
    env = {"NANOPOW_VIRTUAL_DEVICES": "4", "NANOPOW_FAULT_INVALID": "1", "NANOPOW_TEST_HOOKS": "1", "DRIVER_MASK": "0"}
    if binary == "abi_asan_driver":
        env.update(ASAN_OPTIONS="detect_leaks=1:halt_on_error=1:verify_asan_link_order=0", LSAN_OPTIONS="suppressions=tools/lsan.supp")
    else:
        env.update(TSAN_OPTIONS="suppressions=tools/tsan.supp:halt_on_error=1")
    _run(binary, env)


@pytest.mark.gpu
@pytest.mark.parametrize("binary", ["abi_asan_driver", "abi_tsan_driver"])
def test_cpu_workers_under_sanitizers(binary):
    """The pool's CPU workers (npow_cpu.cpp, --cpu-threads) under ASan / TSan: 2 CPU threads as one more
    device, every search, ticket (cancelled ones too) and bounded range over the GPU and the CPU device
    (DRIVER_MASK=0)."""
    env = {"DRIVER_CPU_THREADS": "2", "DRIVER_MASK": "0"}
    if binary == "abi_asan_driver":
        env.update(ASAN_OPTIONS="detect_leaks=1:halt_on_error=1:verify_asan_link_order=0", LSAN_OPTIONS="suppressions=tools/lsan.supp")
    else:
        env.update(TSAN_OPTIONS="suppressions=tools/tsan.supp:halt_on_error=1")
    _run(binary, env)
