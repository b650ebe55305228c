"""ctypes binding of libnanopow.so (the C ABI declared in include/nanopow.h).

The product path has no CPU fallback: if the HIP library is missing, or no
GPU is visible, every entry point here raises :class:`NanoPowError`.  ctypes
releases the GIL for the duration of each foreign call, so searches can run in
worker threads while the HTTP server keeps serving ``work_cancel``
(client/work_handler.py:61-80 sends it on a second connection while a
``work_generate`` is pending).
"""
from __future__ import annotations

import ctypes
import os
import threading
from dataclasses import dataclass
from typing import List, Optional, Sequence, Tuple

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("NANOPOW_LIB", os.path.join(_HERE, "libnanopow.so"))

NPOW_OK = 0
NPOW_CANCELLED = 1
NPOW_EXHAUSTED = 2
NPOW_PENDING = 3
NPOW_ERR_NOT_INITIALISED = -1
NPOW_ERR_NO_DEVICE = -2
NPOW_ERR_BAD_ARGUMENT = -3
NPOW_ERR_HIP = -4
NPOW_ERR_INVALID_WORK = -5
NPOW_ERR_CAPACITY = -6
NPOW_ERR_INTERNAL = -7

NPOW_ABI_VERSION = 6
# hash paths of npow_values_path
NPOW_PATH_SEARCH = 0   # the stream the search and sweep kernels execute (four 512-lane workgroups per CU)
NPOW_PATH_SEQ = 1      # a second generated stream, scheduled without barriers
NPOW_PATH_GENERIC = 2  # plain HIP C++ of the 12 rounds, one (root, nonce) per lane

M64 = (1 << 64) - 1

# Every symbol include/nanopow.h declares (tests/test_abi.py checks the export table).
EXPORTED_SYMBOLS = (
    "npow_init", "npow_shutdown", "npow_last_error", "npow_work_value", "npow_search",
    "npow_search_batch", "npow_sweep", "npow_values", "npow_values_pairs", "npow_set_tuning",
    "npow_device_stats_get", "npow_device_stats_reset", "npow_version",
    "npow_submit", "npow_wait", "npow_cancel", "npow_pool_config", "npow_pool_status",
    "npow_set_pool_tuning", "npow_values_path", "npow_wait_info", "npow_device_stats_get_sized",
    "npow_abi_version", "npow_config_cpu_threads", "npow_wait_result",
)


class NanoPowError(RuntimeError):
    def __init__(self, code: int, message: str):
        super().__init__(f"nanopow error {code}: {message}")
        self.code = code
        self.message = message


class DeviceStats(ctypes.Structure):
    _fields_ = [
        ("launches", ctypes.c_uint64),
        ("nonces", ctypes.c_uint64),
        ("kernel_ms", ctypes.c_double),
        ("invalid_work", ctypes.c_uint64),
        ("cus", ctypes.c_int32),
        ("grid", ctypes.c_int32),
        ("clock_mhz", ctypes.c_double),
        ("host_cpu_ms", ctypes.c_double),
        ("host_wall_ms", ctypes.c_double),
        ("dead", ctypes.c_int32),
        ("pool_groups", ctypes.c_int32),
        ("early_finishes", ctypes.c_uint64),
        ("early_mismatches", ctypes.c_uint64),
        ("yields", ctypes.c_uint64),
        ("dyn_entries", ctypes.c_uint64),
        ("kills_relayed", ctypes.c_uint64),  # ABI 3
        ("late_nonces", ctypes.c_uint64),    # ABI 4
        ("hip_device", ctypes.c_int32),
        ("cu_first", ctypes.c_int32),
        ("idle_ms", ctypes.c_double),        # ABI 5
        ("idle_gaps", ctypes.c_uint64),
        ("affinity_checks", ctypes.c_uint64),
        ("affinity_failures", ctypes.c_uint64),
        ("watcher_decisions", ctypes.c_uint64),
        # ABI 6
        ("stale_drains", ctypes.c_uint64),
        ("linger_ms", ctypes.c_double),
        ("linger_relays", ctypes.c_uint64),
        ("stale_late", ctypes.c_uint64),
        ("stale_missing", ctypes.c_uint64),
        ("stale_gpu_delay_us", ctypes.c_double),
    ]


class SearchInfo(ctypes.Structure):
    """npow_search_info: one search's outcome and host timeline (us since npow_submit)."""
    _fields_ = [
        ("size", ctypes.c_uint32),
        ("status", ctypes.c_int32),
        ("nonce", ctypes.c_uint64),
        ("value", ctypes.c_uint64),
        ("nonces_done", ctypes.c_uint64),
        ("winner_device", ctypes.c_int32),
        ("n_devices", ctypes.c_int32),
        ("decide_us", ctypes.c_double),
        ("finish_us", ctypes.c_double),
        ("stop_after_decide_us", ctypes.c_double),
        ("overshoot_nonces", ctypes.c_uint64),
        ("late_nonces_losers", ctypes.c_uint64),  # ABI 4: counted on the devices
        ("late_nonces_winner", ctypes.c_uint64),
        ("adopt_us", ctypes.c_double),            # ABI 5: host timeline
        ("launch_us", ctypes.c_double),
        ("launch_all_us", ctypes.c_double),
        ("win_seen_us", ctypes.c_double),
    ]


@dataclass
class SweepResult:
    status: int            # NPOW_OK, or NPOW_CANCELLED (hits then holds what was found before it)
    hits: List[int]        # ascending (nonce - start); at most cap of them
    total: int             # exact number of hits (may exceed len(hits) only with status != OK)


@dataclass
class SearchResult:
    status: int            # NPOW_OK / NPOW_CANCELLED / NPOW_EXHAUSTED
    nonce: Optional[int]
    value: Optional[int]
    nonces_done: int


_lib: Optional[ctypes.CDLL] = None
_lib_lock = threading.Lock()


def load(path: str = LIB_PATH) -> ctypes.CDLL:
    """Load libnanopow.so and declare every prototype (no device is touched)."""
    global _lib
    with _lib_lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(path):
            raise NanoPowError(NPOW_ERR_NOT_INITIALISED,
                               f"{path} not built: run `make -C nano-dpow_amd/csrc` "
                               "(or __graft_entry__.build())")
        lib = ctypes.CDLL(path)
        u8p = ctypes.c_char_p
        u64, u32 = ctypes.c_uint64, ctypes.c_uint32
        pu64 = ctypes.POINTER(ctypes.c_uint64)
        p = ctypes.c_void_p
        lib.npow_init.argtypes = [ctypes.POINTER(ctypes.c_int)]
        lib.npow_init.restype = ctypes.c_int
        lib.npow_shutdown.argtypes = []
        lib.npow_shutdown.restype = None
        lib.npow_last_error.argtypes = []
        lib.npow_last_error.restype = ctypes.c_char_p
        lib.npow_version.argtypes = []
        lib.npow_version.restype = ctypes.c_char_p
        lib.npow_work_value.argtypes = [u8p, u64]
        lib.npow_work_value.restype = u64
        lib.npow_search.argtypes = [u8p, u64, u64, u64, u64, p, pu64, pu64, pu64]
        lib.npow_search.restype = ctypes.c_int
        lib.npow_search_batch.argtypes = [u8p, p, u32, u64, u64, p, p, p, p, pu64]
        lib.npow_search_batch.restype = ctypes.c_int
        lib.npow_sweep.argtypes = [u8p, u64, u64, u64, u64, p, p, u64, pu64]
        lib.npow_sweep.restype = ctypes.c_int
        lib.npow_values.argtypes = [ctypes.c_int, u8p, u64, u64, p]
        lib.npow_values.restype = ctypes.c_int
        lib.npow_values_pairs.argtypes = [ctypes.c_int, u8p, p, u32, p]
        lib.npow_values_pairs.restype = ctypes.c_int
        lib.npow_set_tuning.argtypes = [u32, u32, u32]
        lib.npow_set_tuning.restype = ctypes.c_int
        lib.npow_device_stats_get.argtypes = [ctypes.c_int, ctypes.POINTER(DeviceStats)]
        lib.npow_device_stats_get.restype = ctypes.c_int
        lib.npow_device_stats_reset.argtypes = [ctypes.c_int]
        lib.npow_device_stats_reset.restype = ctypes.c_int
        lib.npow_submit.argtypes = [u8p, u64, u64, u64, u64, p, pu64]
        lib.npow_submit.restype = ctypes.c_int
        lib.npow_wait.argtypes = [u64, ctypes.c_int64, pu64, pu64, pu64]
        lib.npow_wait.restype = ctypes.c_int
        lib.npow_cancel.argtypes = [u64]
        lib.npow_cancel.restype = ctypes.c_int
        lib.npow_pool_config.argtypes = [u32]
        lib.npow_pool_config.restype = ctypes.c_int
        lib.npow_pool_status.argtypes = [ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint32)]
        lib.npow_pool_status.restype = ctypes.c_int
        lib.npow_set_pool_tuning.argtypes = [u32, u32]
        lib.npow_set_pool_tuning.restype = ctypes.c_int
        # ABI 3 (a library of an earlier revision, e.g. an A/B build of round-2 sources, lacks them:
        # stats() then falls back to npow_device_stats_get, whose struct is a prefix of DeviceStats)
        if hasattr(lib, "npow_abi_version"):
            lib.npow_values_path.argtypes = [ctypes.c_int, u8p, u64, u64, ctypes.c_int, p]
            lib.npow_values_path.restype = ctypes.c_int
            lib.npow_wait_info.argtypes = [u64, ctypes.c_int64, ctypes.POINTER(SearchInfo)]
            lib.npow_wait_info.restype = ctypes.c_int
            lib.npow_device_stats_get_sized.argtypes = [ctypes.c_int, ctypes.POINTER(DeviceStats), u64]
            lib.npow_device_stats_get_sized.restype = ctypes.c_int
            lib.npow_abi_version.argtypes = []
            lib.npow_abi_version.restype = ctypes.c_int
        if hasattr(lib, "npow_config_cpu_threads"):  # ABI 4
            lib.npow_config_cpu_threads.argtypes = [u32]
            lib.npow_config_cpu_threads.restype = ctypes.c_int
            lib.npow_wait_result.argtypes = [u64, ctypes.c_int64, pu64, pu64]
            lib.npow_wait_result.restype = ctypes.c_int
        _lib = lib
        return lib


def _check(rc: int, lib: ctypes.CDLL, ok=(NPOW_OK,)) -> int:
    if rc in ok:
        return rc
    msg = lib.npow_last_error()
    raise NanoPowError(rc, msg.decode("utf-8", "replace") if msg else "")


def _root(root: bytes) -> bytes:
    if not isinstance(root, (bytes, bytearray)) or len(root) != 32:
        raise ValueError("root must be 32 bytes")
    return bytes(root)


class CancelToken:
    """A caller-owned 32-bit word the engine polls; set() stops a running search."""

    def __init__(self) -> None:
        self._word = ctypes.c_uint32(0)

    def set(self) -> None:
        self._word.value = 1

    def clear(self) -> None:
        self._word.value = 0

    @property
    def is_set(self) -> bool:
        return bool(self._word.value)

    @property
    def address(self) -> int:
        return ctypes.addressof(self._word)


_ORPHANED_CANCEL_WORDS: list = []


class Ticket:
    """A submitted search (npow_submit); wait() returns its SearchResult once."""

    def __init__(self, engine: "Engine", ticket: int, cancel: Optional[CancelToken]) -> None:
        self.engine = engine
        self.ticket = ticket
        self.cancel_token = cancel  # keeps the cancel word alive while the engine may read it
        self.result: Optional[SearchResult] = None

    def wait(self, timeout: Optional[float] = None) -> Optional[SearchResult]:
        """Block until the search ends (timeout None) or up to `timeout` seconds; None if
        it is still running then."""
        if self.result is not None:
            return self.result
        lib = self.engine.lib
        nonce, value, done = ctypes.c_uint64(0), ctypes.c_uint64(0), ctypes.c_uint64(0)
        us = -1 if timeout is None else max(0, int(timeout * 1e6))
        rc = lib.npow_wait(self.ticket, us, ctypes.byref(nonce), ctypes.byref(value), ctypes.byref(done))
        if rc == NPOW_PENDING:
            return None
        self.cancel_token = None
        _check(rc, lib, ok=(NPOW_OK, NPOW_CANCELLED, NPOW_EXHAUSTED))
        self.result = (SearchResult(rc, nonce.value, value.value, done.value) if rc == NPOW_OK
                       else SearchResult(rc, None, None, done.value))
        return self.result

    def wait_result(self, timeout: Optional[float] = None) -> Optional[SearchResult]:
        """The search's outcome as soon as it is known (npow_wait_result: the winner accepted, the cancellation
        seen), before the other devices of a split search have stopped; None if still running after `timeout`
        seconds.  nonces_done is 0 here: wait() or wait_info() must still collect the ticket."""
        if self.result is not None:
            return self.result
        lib = self.engine.lib
        nonce, value = ctypes.c_uint64(0), ctypes.c_uint64(0)
        us = -1 if timeout is None else max(0, int(timeout * 1e6))
        rc = lib.npow_wait_result(self.ticket, us, ctypes.byref(nonce), ctypes.byref(value))
        if rc == NPOW_PENDING:
            return None
        _check(rc, lib, ok=(NPOW_OK, NPOW_CANCELLED, NPOW_EXHAUSTED))
        return (SearchResult(rc, nonce.value, value.value, 0) if rc == NPOW_OK
                else SearchResult(rc, None, None, 0))

    def wait_info(self, timeout: Optional[float] = None) -> Optional[SearchInfo]:
        """wait() with the search's timeline (npow_wait_info): winner device, host times of the
        decision and the finish, and the other devices' overshoot after the decision.  None if
        still running after `timeout` seconds."""
        if self.result is not None:
            raise RuntimeError("the ticket's result was already collected")
        lib = self.engine.lib
        info = SearchInfo()
        info.size = ctypes.sizeof(SearchInfo)
        us = -1 if timeout is None else max(0, int(timeout * 1e6))
        rc = lib.npow_wait_info(self.ticket, us, ctypes.byref(info))
        if rc == NPOW_PENDING:
            return None
        self.cancel_token = None
        _check(rc, lib, ok=(NPOW_OK, NPOW_CANCELLED, NPOW_EXHAUSTED))
        self.result = (SearchResult(rc, info.nonce, info.value, info.nonces_done) if rc == NPOW_OK
                       else SearchResult(rc, None, None, info.nonces_done))
        return info

    def cancel(self) -> None:
        if self.result is None:
            _check(self.engine.lib.npow_cancel(self.ticket), self.engine.lib)

    def __del__(self) -> None:
        # An abandoned ticket: cancel its search and collect it, so the engine forgets the job
        # and stops reading this ticket's cancel word before that word is freed.  A job that
        # does not end within 10 s keeps its cancel word alive for the life of the process.
        if self.result is not None or not getattr(self, "ticket", 0):
            return
        try:
            lib = self.engine.lib
            lib.npow_cancel(self.ticket)
            if lib.npow_wait(self.ticket, 10_000_000, None, None, None) == NPOW_PENDING:
                _ORPHANED_CANCEL_WORDS.append(self.cancel_token)
        except Exception:  # interpreter shutdown: the library may already be gone
            pass


class Engine:
    """Thin object wrapper over the C ABI (one per process is enough)."""

    def __init__(self, path: str = LIB_PATH, cpu_threads: int = 0) -> None:
        """cpu_threads > 0: add that many CPU worker threads as one more logical device after the GPUs
        (npow_config_cpu_threads; the reference work server's --cpu-threads).  npow_init is process-wide:
        asking for CPU threads once the engine is initialised in this process raises NanoPowError
        (NPOW_ERR_BAD_ARGUMENT), as npow_config_cpu_threads must precede npow_init."""
        self.lib = load(path)
        if cpu_threads:
            _check(self.lib.npow_config_cpu_threads(cpu_threads), self.lib)
        n = ctypes.c_int(0)
        _check(self.lib.npow_init(ctypes.byref(n)), self.lib)
        self.n_devices = n.value
        self.cpu_device = None  # logical id of the CPU workers' device, if any
        for d in range(self.n_devices):
            if self.stats(d).hip_device < 0:
                self.cpu_device = d
        self.gpu_mask = ((1 << self.n_devices) - 1) & ~(0 if self.cpu_device is None else 1 << self.cpu_device)

    # -- CPU helpers -------------------------------------------------------------------
    def work_value(self, root: bytes, nonce: int) -> int:
        return int(self.lib.npow_work_value(_root(root), nonce & M64))

    # -- GPU paths ---------------------------------------------------------------------
    def search(self, root: bytes, threshold: int, start: int = 0, device_mask: int = 0,
               max_nonces_per_device: int = 0, cancel: Optional[CancelToken] = None) -> SearchResult:
        nonce = ctypes.c_uint64(0)
        value = ctypes.c_uint64(0)
        done = ctypes.c_uint64(0)
        rc = self.lib.npow_search(_root(root), threshold & M64, start & M64, device_mask,
                                  max_nonces_per_device, cancel.address if cancel else None,
                                  ctypes.byref(nonce), ctypes.byref(value), ctypes.byref(done))
        _check(rc, self.lib, ok=(NPOW_OK, NPOW_CANCELLED, NPOW_EXHAUSTED))
        if rc == NPOW_OK:
            return SearchResult(rc, nonce.value, value.value, done.value)
        return SearchResult(rc, None, None, done.value)

    # -- work pool: asynchronous searches ---------------------------------------------------
    def submit(self, root: bytes, threshold: int, start: int = 0, device_mask: int = 0,
               max_nonces_per_device: int = 0, cancel: Optional[CancelToken] = None) -> "Ticket":
        """Queue a first-win search and return at once (npow_submit).  Keep `cancel` alive
        until the ticket's result has been collected (the Ticket holds a reference)."""
        t = ctypes.c_uint64(0)
        _check(self.lib.npow_submit(_root(root), threshold & M64, start & M64, device_mask, max_nonces_per_device,
                                    cancel.address if cancel else None, ctypes.byref(t)), self.lib)
        return Ticket(self, t.value, cancel)

    def pool_config(self, max_active: int) -> None:
        _check(self.lib.npow_pool_config(max_active), self.lib)

    def pool_status(self) -> Tuple[int, int]:
        q, a = ctypes.c_uint32(0), ctypes.c_uint32(0)
        _check(self.lib.npow_pool_status(ctypes.byref(q), ctypes.byref(a)), self.lib)
        return q.value, a.value

    def search_batch(self, roots: Sequence[bytes], thresholds: Sequence[int], device_mask: int = 0,
                     max_nonces_per_root: int = 0,
                     cancels: Optional[Sequence[Optional[CancelToken]]] = None) -> Tuple[List[SearchResult], int]:
        n = len(roots)
        if len(thresholds) != n:
            raise ValueError("roots and thresholds differ in length")
        rb = b"".join(_root(r) for r in roots)
        th = (ctypes.c_uint64 * n)(*[t & M64 for t in thresholds])
        nonces = (ctypes.c_uint64 * n)()
        values = (ctypes.c_uint64 * n)()
        status = (ctypes.c_int32 * n)()
        done = ctypes.c_uint64(0)
        cptr = None
        if cancels is not None:
            arr = (ctypes.c_void_p * n)(*[(c.address if c else None) for c in cancels])
            cptr = ctypes.addressof(arr)
        rc = self.lib.npow_search_batch(rb, ctypes.addressof(th), n, device_mask, max_nonces_per_root, cptr,
                                        ctypes.addressof(nonces), ctypes.addressof(values),
                                        ctypes.addressof(status), ctypes.byref(done))
        _check(rc, self.lib)
        out = []
        for i in range(n):
            if status[i] == NPOW_OK:
                out.append(SearchResult(NPOW_OK, nonces[i], values[i], 0))
            else:
                out.append(SearchResult(status[i], None, None, 0))
        return out, done.value

    def sweep_result(self, root: bytes, threshold: int, start: int, count: int, device_mask: int = 0,
                     cap: int = 1 << 16, cancel: Optional[CancelToken] = None) -> SweepResult:
        """npow_sweep with its status: a cancelled sweep returns status NPOW_CANCELLED and the
        hits found so far, never mistakable for the exact hit set of the range."""
        out = (ctypes.c_uint64 * max(cap, 1))()
        n = ctypes.c_uint64(0)
        rc = self.lib.npow_sweep(_root(root), threshold & M64, start & M64, count, device_mask,
                                 cancel.address if cancel else None, ctypes.addressof(out), cap,
                                 ctypes.byref(n))
        _check(rc, self.lib, ok=(NPOW_OK, NPOW_CANCELLED))
        return SweepResult(rc, list(out[: min(n.value, cap)]), n.value)

    def sweep(self, root: bytes, threshold: int, start: int, count: int, device_mask: int = 0,
              cap: int = 1 << 16, cancel: Optional[CancelToken] = None) -> List[int]:
        """Every hit of [start, start + count) (exact).  Raises NanoPowError(NPOW_CANCELLED) if
        `cancel` stopped it (sweep_result() returns the partial hits with the status)."""
        r = self.sweep_result(root, threshold, start, count, device_mask, cap, cancel)
        if r.status != NPOW_OK:
            raise NanoPowError(r.status, f"sweep cancelled after {r.total} hits: the hit set is partial")
        return r.hits

    def values(self, root: bytes, start: int, count: int, device: int = 0, path: Optional[int] = None) -> List[int]:
        """Work values of start .. start + count - 1: npow_values (the search kernels' stream), or
        npow_values_path with an NPOW_PATH_* constant."""
        out = (ctypes.c_uint64 * max(count, 1))()
        if path is None:
            rc = self.lib.npow_values(device, _root(root), start & M64, count, ctypes.addressof(out))
        else:
            rc = self.lib.npow_values_path(device, _root(root), start & M64, count, path, ctypes.addressof(out))
        _check(rc, self.lib)
        return list(out[:count])

    def values_array(self, root: bytes, start: int, count: int, device: int = 0, path: int = NPOW_PATH_SEARCH):
        """The same as values() into a numpy uint64 array (large ranges)."""
        import numpy as np
        out = np.empty(max(count, 1), dtype=np.uint64)
        _check(self.lib.npow_values_path(device, _root(root), start & M64, count, path, out.ctypes.data), self.lib)
        return out[:count]

    def values_pairs(self, roots: Sequence[bytes], nonces: Sequence[int], device: int = 0) -> List[int]:
        n = len(nonces)
        if len(roots) != n:  # the library reads n * 32 root bytes
            raise ValueError(f"{len(roots)} roots for {n} nonces")
        rb = b"".join(_root(r) for r in roots)
        nn = (ctypes.c_uint64 * max(n, 1))(*[x & M64 for x in nonces])
        out = (ctypes.c_uint64 * max(n, 1))()
        _check(self.lib.npow_values_pairs(device, rb, ctypes.addressof(nn), n, ctypes.addressof(out)), self.lib)
        return list(out[:n])

    def set_tuning(self, iters_per_launch: int = 0, poll_interval: int = 0, blocks_per_cu: int = 0) -> None:
        _check(self.lib.npow_set_tuning(iters_per_launch, poll_interval, blocks_per_cu), self.lib)

    def set_pool_tuning(self, budget_us: Optional[int] = None, blocks_per_cu: int = 0) -> None:
        """Search launches: time budget in us (0 = off, None keeps) and workgroups per CU (0 keeps)."""
        _check(self.lib.npow_set_pool_tuning(0xffffffff if budget_us is None else budget_us, blocks_per_cu),
               self.lib)

    def set_launch_budget(self, budget_us: int) -> None:
        self.set_pool_tuning(budget_us=budget_us)

    def stats(self, device: int = 0) -> DeviceStats:
        s = DeviceStats()
        if hasattr(self.lib, "npow_device_stats_get_sized"):
            _check(self.lib.npow_device_stats_get_sized(device, ctypes.byref(s), ctypes.sizeof(s)), self.lib)
        else:
            _check(self.lib.npow_device_stats_get(device, ctypes.byref(s)), self.lib)
        return s

    def abi_version(self) -> int:
        return int(self.lib.npow_abi_version())

    def reset_stats(self, device: int = 0) -> None:
        _check(self.lib.npow_device_stats_reset(device), self.lib)

    def version(self) -> str:
        return self.lib.npow_version().decode()


_engine: Optional[Engine] = None
_engine_lock = threading.Lock()


def engine(cpu_threads: int = 0) -> Engine:
    """Process-wide engine (initialised on first use; raises if no GPU).  cpu_threads: CPU workers
    beside the GPUs (Engine), honoured by the first call only."""
    global _engine
    with _engine_lock:
        if _engine is None:
            _engine = Engine(cpu_threads=cpu_threads)
        return _engine
