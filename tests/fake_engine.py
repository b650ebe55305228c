"""CPU stand-in for libnanopow's Engine, built on the oracle (TEST INFRASTRUCTURE).

Lets the work-server logic (queueing, cancel, JSON surface) be tested without
a GPU.  It is never importable from the product package: the product's engine
is libnanopow.so only.
"""
import threading
import time
from types import SimpleNamespace

import oracle
from nanopow._lib import NPOW_CANCELLED, NPOW_EXHAUSTED, NPOW_OK, SearchResult


class _Flag:
    def __init__(self):
        self.is_set = False


class _Ticket:
    def __init__(self, fn):
        self._ev = threading.Event()
        self._res = None
        self._info = None

        def run():
            out = fn()
            self._res, self._info = out if isinstance(out, tuple) else (out, None)
            self._ev.set()
        threading.Thread(target=run, daemon=True).start()

    def wait(self, timeout=None):
        return self._res if self._ev.wait(timeout) else None

    def cancel(self):
        self._own.is_set = True

    def wait_result(self, timeout=None):  # the engine's npow_wait_result; here the outcome is the final result
        return self.wait(timeout)

    def wait_info(self, timeout=None):
        if not self._ev.wait(timeout):
            return None
        r, info = self._res, self._info
        return info or SimpleNamespace(status=r.status, nonce=r.nonce, value=r.value, nonces_done=r.nonces_done,
                                       winner_device=0, n_devices=1, decide_us=0.0, finish_us=0.0,
                                       stop_after_decide_us=0.0, overshoot_nonces=0, late_nonces_losers=0, late_nonces_winner=0,
                                       adopt_us=0.0, launch_us=0.0, launch_all_us=0.0, win_seen_us=0.0)


class OracleEngine:
    """n_devices > 1 emulates the pool's multi-device split: a search over a mask of G devices runs G
    threads on the disjoint strides start + k * 2^64 / G, the first win stopping the others."""

    def __init__(self, chunk=1 << 12, delay=0.0, n_devices=1):
        self.chunk = chunk
        self.delay = delay
        self.n_devices = n_devices
        self.calls = []
        self.lock = threading.Lock()
        self._stats = [dict(nonces=0, launches=0, kernel_ms=0.0) for _ in range(n_devices)]
        self.cpu_device, self.gpu_mask = None, (1 << n_devices) - 1

    def stats(self, device=0):
        st = self._stats[device]
        return SimpleNamespace(kernel_ms=st["kernel_ms"], nonces=st["nonces"], launches=st["launches"],
                               clock_mhz=0.0, early_finishes=0, kills_relayed=0, host_cpu_ms=0.0,
                               host_wall_ms=1.0, grid=0, pool_groups=4, late_nonces=0, hip_device=0,
                               cu_first=-1, cus=256, idle_ms=0.0, idle_gaps=0, affinity_checks=0, affinity_failures=0,
                               watcher_decisions=0, dyn_entries=0, stale_drains=0, linger_ms=0.0, linger_relays=0,
                               stale_late=0, stale_missing=0, stale_gpu_delay_us=0.0)

    def version(self):
        return "oracle stand-in engine (tests/fake_engine.py)"

    def reset_stats(self, device=0):
        self._stats[device] = dict(nonces=0, launches=0, kernel_ms=0.0)

    def _split(self, root, threshold, start, device_mask, cancel):
        devs = [d for d in range(self.n_devices) if device_mask == 0 or (device_mask >> d) & 1]
        G = len(devs)
        spacing = (1 << 64) // G
        stop = _Flag()
        out = [None] * G
        t0 = time.perf_counter()
        decided = [None]

        def run(k):
            t = time.perf_counter()
            r = self.search(root, threshold, (start + k * spacing) % (1 << 64), cancel=_Either(stop, cancel))
            with self.lock:
                st = self._stats[devs[k]]
                st["nonces"] += r.nonces_done
                st["launches"] += 1
                st["kernel_ms"] += (time.perf_counter() - t) * 1e3
                if r.status == NPOW_OK and decided[0] is None:
                    decided[0] = (k, time.perf_counter())
                    stop.is_set = True
            out[k] = (r, time.perf_counter())
        ths = [threading.Thread(target=run, args=(k,)) for k in range(G)]
        for t in ths:
            t.start()
        for t in ths:
            t.join()
        done = sum(r.nonces_done for r, _ in out)
        if decided[0] is None:
            res = SearchResult(out[0][0].status, None, None, done)
            return res, None
        k, td = decided[0]
        win = out[k][0]
        spans = [max(0.0, (te - td) * 1e6) for j, (_, te) in enumerate(out) if j != k]
        res = SearchResult(NPOW_OK, win.nonce, win.value, done)
        info = SimpleNamespace(status=NPOW_OK, nonce=win.nonce, value=win.value, nonces_done=done,
                               winner_device=devs[k], n_devices=G, decide_us=(td - t0) * 1e6,
                               finish_us=(max(te for _, te in out) - t0) * 1e6,
                               stop_after_decide_us=max(spans, default=0.0), overshoot_nonces=0, late_nonces_losers=0, late_nonces_winner=0,
                               adopt_us=0.0, launch_us=0.0, launch_all_us=0.0, win_seen_us=(td - t0) * 1e6)
        return res, info

    def work_value(self, root, nonce):
        return oracle.work_value(root, nonce)

    def search(self, root, threshold, start=0, device_mask=0, max_nonces_per_device=0, cancel=None):
        with self.lock:
            self.calls.append((root, threshold, start))
        done = 0
        n = start
        while True:
            if cancel is not None and cancel.is_set:
                return SearchResult(NPOW_CANCELLED, None, None, done)
            cnt = self.chunk if not max_nonces_per_device else min(self.chunk, max_nonces_per_device - done)
            if cnt <= 0:
                return SearchResult(NPOW_EXHAUSTED, None, None, done)
            scanned, found = oracle.search(root, threshold, n, cnt)
            done += scanned
            if found is not None:
                return SearchResult(NPOW_OK, found, oracle.work_value(root, found), done)
            n += cnt
            if self.delay:
                time.sleep(self.delay)

    def submit(self, root, threshold, start=0, device_mask=0, max_nonces_per_device=0, cancel=None):
        own = _Flag()  # Ticket.cancel() (npow_cancel)
        either = _Either(own, cancel)
        if self.n_devices > 1 and not max_nonces_per_device:
            tk = _Ticket(lambda: self._split(root, threshold, start, device_mask, either))
        else:
            tk = _Ticket(lambda: self.search(root, threshold, start, device_mask, max_nonces_per_device, either))
        tk._own = own
        return tk


class _Either:
    def __init__(self, a, b):
        self.a, self.b = a, b

    @property
    def is_set(self):
        return self.a.is_set or (self.b is not None and self.b.is_set)
