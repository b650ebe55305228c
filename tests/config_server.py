"""Child process of tests/test_gpu_configs.py: the JSON work server (nanopow.server.HttpWorkServer)
on libnanopow, opened with NANOPOW_VIRTUAL_DEVICES logical devices so that every request is split
over that many disjoint strides.  The engine is wrapped only to record each search's nonces_done
(the JSON reply does not carry it), so the parent can check the per-job accounting against the
device counters.

Protocol (stdout / stdin, one JSON line each):
  -> {"address": "127.0.0.1:PORT", "devices": G}        once the server listens
  <- "stats"                                              after the parent's burst
  -> {"job_nonces": sum of nonces_done over every search, "device_nonces": [per device],
      "launches": [per device], "searches": n}
Then it stops the server and exits."""
import json
import os
import sys
import threading

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "nano-dpow_amd"))

from nanopow import _lib  # noqa: E402
from nanopow.server import HttpWorkServer, WorkServer  # noqa: E402


class CountingEngine:
    """libnanopow's Engine, recording nonces_done of every collected search."""

    def __init__(self, eng):
        self.eng = eng
        self.n_devices = eng.n_devices
        self.lock = threading.Lock()
        self.nonces = 0
        self.searches = 0

    def work_value(self, root, nonce):
        return self.eng.work_value(root, nonce)

    def submit(self, *a, **kw):
        t = self.eng.submit(*a, **kw)
        outer = self

        class _T:
            def wait(self, timeout=None):
                r = t.wait(timeout)
                if r is not None:
                    with outer.lock:
                        outer.nonces += r.nonces_done
                        outer.searches += 1
                return r
        return _T()


def main():
    eng = _lib.Engine()
    G = eng.n_devices
    for d in range(G):
        eng.reset_stats(d)
    ce = CountingEngine(eng)
    max_active = int(os.environ.get("CONFIG_MAX_ACTIVE", "64"))
    srv = HttpWorkServer(WorkServer(ce, max_active=max_active, device_mask=0), "127.0.0.1", 0).start()
    print(json.dumps({"address": srv.address, "devices": G}), flush=True)
    for line in sys.stdin:
        if line.strip() == "stats":
            break
    srv.stop()
    st = [eng.stats(d) for d in range(G)]
    print(json.dumps({"job_nonces": ce.nonces, "searches": ce.searches,
                      "device_nonces": [s.nonces for s in st], "launches": [s.launches for s in st],
                      "kernel_ms": [s.kernel_ms for s in st]}), flush=True)


if __name__ == "__main__":
    main()
