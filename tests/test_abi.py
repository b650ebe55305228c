"""The C ABI library: loads, exports every symbol include/nanopow.h declares, CPU entry points.

No GPU compute here (CPU suite); tests/test_gpu_parity.py covers the kernels.
"""
import ctypes
import os
import re
import subprocess

import pytest

from conftest import ROOT, load_golden
from nanopow import _lib

HEADER = os.path.join(ROOT, "include", "nanopow.h")


def declared_symbols():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(npow_[a-z_]+)\s*\(", txt)))


def test_library_built_in_tree():
    assert os.path.exists(_lib.LIB_PATH), "run __graft_entry__.build() / make -C nano-dpow_amd/csrc"


def test_exports_every_declared_symbol():
    syms = declared_symbols()
    assert len(syms) >= 13
    assert sorted(syms) == sorted(_lib.EXPORTED_SYMBOLS)
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r" T (npow_\w+)$", out, flags=re.M))
    missing = set(syms) - exported
    assert not missing, missing
    lib = _lib.load()
    for s in syms:
        assert hasattr(lib, s)


def test_gfx950_code_object_embedded():
    # the fat binary carries an amdgcn-amd-amdhsa--gfx950 code object (no other target)
    blob = open(_lib.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob
    assert not re.search(rb"amdgcn-amd-amdhsa--gfx9[0-4]\d", blob)


def test_cpu_work_value_matches_golden():
    lib = _lib.load()
    g = load_golden("work_values.json")["triples"]
    for r, n, v in g:
        assert lib.npow_work_value(bytes.fromhex(r), int(n, 16)) == int(v, 16)


def test_version_string():
    assert b"gfx950" in _lib.load().npow_version()


def test_uninitialised_calls_fail_cleanly():
    lib = _lib.load()
    out = ctypes.c_uint64(0)
    # search before npow_init (or without a GPU) must return an error, never fall back to the CPU
    rc = lib.npow_search(b"\x00" * 32, 0, 0, 0, 0, None, ctypes.byref(out), None, None)
    assert rc < 0
    assert lib.npow_last_error()


def test_stats_reject_null_out():
    """npow_device_stats_get / _sized with out == NULL (or size 0) return
    NPOW_ERR_BAD_ARGUMENT instead of writing through the pointer."""
    lib = _lib.load()
    assert lib.npow_device_stats_get(0, None) == _lib.NPOW_ERR_BAD_ARGUMENT
    assert lib.npow_device_stats_get_sized(0, None, ctypes.sizeof(_lib.DeviceStats)) == _lib.NPOW_ERR_BAD_ARGUMENT
    st = _lib.DeviceStats()
    assert lib.npow_device_stats_get_sized(0, ctypes.byref(st), 0) == _lib.NPOW_ERR_BAD_ARGUMENT
    assert lib.npow_last_error()


def test_init_without_gpu_reports_no_device():
    import torch  # noqa: F401  (only to ask whether this host has a GPU)
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    n = ctypes.c_int(-1)
    rc = _lib.load().npow_init(ctypes.byref(n))
    assert rc == _lib.NPOW_ERR_NO_DEVICE
    with pytest.raises(_lib.NanoPowError):
        _lib.Engine()


@pytest.mark.parametrize("cname,pytype", [("npow_device_stats", "DeviceStats"), ("npow_search_info", "SearchInfo")])
def test_struct_layout_matches_header(tmp_path, cname, pytype):
    """The ctypes mirrors of npow_device_stats and npow_search_info (_lib.DeviceStats, _lib.SearchInfo)
    have the C structs' sizes and field offsets: compiled from include/nanopow.h with gcc and compared
    field by field."""
    cls = getattr(_lib, pytype)
    fields = [f for f, _ in cls._fields_]
    src = tmp_path / "layout.c"
    src.write_text('#include <stddef.h>\n#include <stdio.h>\n#include "nanopow.h"\nint main(void) {\n'
                   f'  printf("%zu\\n", sizeof({cname}));\n'
                   + "".join(f'  printf("%zu\\n", offsetof({cname}, {f}));\n' for f in fields)
                   + "  return 0;\n}\n")
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), "-o", str(exe), str(src)], check=True)
    vals = [int(x) for x in subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()]
    assert vals[0] == ctypes.sizeof(cls)
    assert vals[1:] == [getattr(cls, f).offset for f in fields]


def test_abi_version_constant_matches_header():
    txt = open(os.path.join(ROOT, "include", "nanopow.h")).read()
    assert re.search(r"#define NPOW_ABI_VERSION (\d+)", txt).group(1) == str(_lib.NPOW_ABI_VERSION)
    for name in ("NPOW_PATH_SEARCH", "NPOW_PATH_SEQ", "NPOW_PATH_GENERIC"):
        assert int(re.search(rf"#define {name} (\d+)", txt).group(1)) == getattr(_lib, name)
    assert _lib.load().npow_abi_version() == _lib.NPOW_ABI_VERSION
