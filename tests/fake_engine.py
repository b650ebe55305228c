"""CPU stand-in for libnanopow's Engine, built on the oracle (TEST INFRASTRUCTURE).

Lets the work-server logic (queueing, cancel, JSON surface) be tested without
a GPU.  It is never importable from the product package: the product's engine
is libnanopow.so only.
"""
import threading
import time

import oracle
from nanopow._lib import NPOW_CANCELLED, NPOW_EXHAUSTED, NPOW_OK, SearchResult


class _Ticket:
    def __init__(self, fn):
        self._ev = threading.Event()
        self._res = None

        def run():
            self._res = fn()
            self._ev.set()
        threading.Thread(target=run, daemon=True).start()

    def wait(self, timeout=None):
        return self._res if self._ev.wait(timeout) else None


class OracleEngine:
    n_devices = 1

    def __init__(self, chunk=1 << 12, delay=0.0):
        self.chunk = chunk
        self.delay = delay
        self.calls = []
        self.lock = threading.Lock()

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
        return _Ticket(lambda: self.search(root, threshold, start, device_mask, max_nonces_per_device, cancel))
