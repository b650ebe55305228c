"""oracle/oracle.py -- TEST INFRASTRUCTURE ONLY (the parity checker).

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import this module.  The product package (``nano-dpow_amd/nanopow``)
never imports it; its work values come from ``libnanopow.so`` alone.

Two independent CPU restatements of the reference's proof-of-work value
(``value = LE_u64(blake2b(LE64(nonce) || root, digest_size=8))``, valid iff
``value >= threshold``; nano-work-server.exe @1661643 ``nano_work``,
server/dpow_server.py:130,296,365,368 ``nanolib.validate_work``):

* :func:`work_value_hashlib` -- Python's stdlib ``hashlib.blake2b`` (the
  reference CPU path named by BASELINE.json ``north_star``).
* :func:`work_value` / :func:`sweep` -- ``oracle/liboracle.so``, a generic
  RFC 7693 BLAKE2b in plain C (``oracle/blake2b_oracle.c``), fast enough for
  exhaustive sweeps.  Pinned against hashlib and the committed fixtures by
  ``tests/test_oracle.py``.
"""
from __future__ import annotations

import ctypes
import hashlib
import os
import subprocess
from typing import List, Optional, Sequence

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liboracle.so")
_lib: Optional[ctypes.CDLL] = None


def build() -> str:
    """Compile oracle/liboracle.so (gcc) if missing or stale."""
    src = os.path.join(_HERE, "blake2b_oracle.c")
    if not os.path.exists(_LIB_PATH) or os.path.getmtime(_LIB_PATH) < os.path.getmtime(src):
        subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def _load() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        build()
        lib = ctypes.CDLL(_LIB_PATH)
        u64, p = ctypes.c_uint64, ctypes.c_void_p
        lib.oracle_work_value.restype = u64
        lib.oracle_work_value.argtypes = [ctypes.c_char_p, u64]
        lib.oracle_work_values.restype = None
        lib.oracle_work_values.argtypes = [ctypes.c_char_p, p, p, ctypes.c_size_t]
        lib.oracle_blake2b.restype = ctypes.c_int
        lib.oracle_blake2b.argtypes = [p, ctypes.c_size_t, ctypes.c_char_p, ctypes.c_size_t]
        lib.oracle_sweep.restype = u64
        lib.oracle_sweep.argtypes = [ctypes.c_char_p, u64, u64, u64, p, u64, ctypes.c_int]
        lib.oracle_values_range.restype = ctypes.c_int
        lib.oracle_values_range.argtypes = [ctypes.c_char_p, u64, u64, p, ctypes.c_int]
        lib.oracle_search.restype = u64
        lib.oracle_search.argtypes = [ctypes.c_char_p, u64, u64, u64,
                                      ctypes.POINTER(u64), ctypes.POINTER(ctypes.c_int)]
        _lib = lib
    return _lib


M64 = (1 << 64) - 1


def work_value_hashlib(root: bytes, nonce: int) -> int:
    """hashlib.blake2b(digest_size=8) over LE64(nonce) || root, read little-endian."""
    assert len(root) == 32
    d = hashlib.blake2b((nonce & M64).to_bytes(8, "little") + root, digest_size=8).digest()
    return int.from_bytes(d, "little")


def blake2b(data: bytes, outlen: int = 64) -> bytes:
    """Generic BLAKE2b through the C restatement (for RFC 7693 self-tests)."""
    out = ctypes.create_string_buffer(outlen)
    rc = _load().oracle_blake2b(out, outlen, data, len(data))
    if rc:
        raise ValueError("bad outlen")
    return out.raw


def work_value(root: bytes, nonce: int) -> int:
    assert len(root) == 32
    return int(_load().oracle_work_value(root, nonce & M64))


def work_values(roots: Sequence[bytes], nonces: Sequence[int]) -> List[int]:
    n = len(nonces)
    assert len(roots) == n
    rb = b"".join(roots)
    nn = (ctypes.c_uint64 * n)(*[x & M64 for x in nonces])
    out = (ctypes.c_uint64 * n)()
    _load().oracle_work_values(rb, ctypes.addressof(nn), ctypes.addressof(out), n)
    return list(out)


def work_values_range(root: bytes, start: int, count: int, threads: Optional[int] = None):
    """numpy uint64 array of the work values of nonces start .. start + count - 1 (mod 2^64), on
    `threads` pthreads (default: every CPU, at most 16)."""
    import numpy as np
    assert len(root) == 32
    if threads is None:
        threads = min(16, os.cpu_count() or 1)
    out = np.empty(count, dtype=np.uint64)
    if count and _load().oracle_values_range(root, start & M64, count, out.ctypes.data, threads) != 0:
        raise MemoryError("oracle_values_range allocation failed")
    return out


def sweep(root: bytes, threshold: int, start: int, count: int, threads: Optional[int] = None,
          cap: int = 1 << 20) -> List[int]:
    """Every nonce in [start, start+count) (mod 2^64) whose value >= threshold, ascending by offset."""
    if threads is None:
        threads = os.cpu_count() or 1
    out = (ctypes.c_uint64 * cap)()
    n = _load().oracle_sweep(root, threshold & M64, start & M64, count, ctypes.addressof(out), cap, threads)
    if n == M64:
        raise MemoryError("oracle_sweep allocation failed")
    if n > cap:
        raise OverflowError(f"{n} hits exceed cap {cap}")
    return list(out[:n])


def search(root: bytes, threshold: int, start: int, max_count: int):
    """Scalar first-win scan (CPU baseline leg). Returns (scanned, nonce or None)."""
    fn = ctypes.c_uint64(0)
    found = ctypes.c_int(0)
    scanned = _load().oracle_search(root, threshold & M64, start & M64, max_count,
                                    ctypes.byref(fn), ctypes.byref(found))
    return int(scanned), (int(fn.value) if found.value else None)
