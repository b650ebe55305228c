#!/usr/bin/env python3
"""JSON-boundary overhead of the work server, without a GPU: an engine whose searches end at once
(submit -> a ticket that is already done) behind HttpWorkServer, driven by a keep-alive HTTP/1.1
client (one connection for every request, as the DPoW client's aiohttp session does,
client/work_handler.py:98-108) and by a new connection per request (urllib).  Prints p50 / p99
round-trip times: what the HTTP + JSON + dispatch layer adds to a search's C-ABI time.

python3 tools/http_overhead.py [n]"""
import http.client
import json
import os
import statistics
import sys
import time
import urllib.request

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "nano-dpow_amd"))
from nanopow._lib import NPOW_OK, SearchResult  # noqa: E402
from nanopow.server import HttpWorkServer, WorkServer  # noqa: E402


class _Done:
    def __init__(self, r):
        self.r = r

    def wait(self, timeout=None):
        return self.r


class InstantEngine:
    n_devices = 1

    def submit(self, root, threshold, start=0, device_mask=0, max_nonces_per_device=0, cancel=None):
        return _Done(SearchResult(NPOW_OK, 0x1234, 0xfffffff900000000, 1))

    def work_value(self, root, nonce):
        return 0xfffffff900000000


def pct(xs, p):
    xs = sorted(xs)
    return xs[min(len(xs) - 1, int(round(p / 100 * (len(xs) - 1))))]


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 3000
    srv = HttpWorkServer(WorkServer(InstantEngine(), max_active=1), "127.0.0.1", 0).start()
    host, port = srv.address.split(":")
    out = {}
    try:
        conn = http.client.HTTPConnection(host, int(port))
        lat = []
        for i in range(n + 200):
            body = json.dumps({"action": "work_generate", "hash": f"{i:064X}", "difficulty": "fffffff800000000"})
            t = time.perf_counter()
            conn.request("POST", "/", body, {"Content-Type": "application/json"})
            rep = json.loads(conn.getresponse().read())
            if i >= 200:
                lat.append(time.perf_counter() - t)
            assert rep["work"] == "0000000000001234"
        conn.close()
        out["keepalive_us"] = {"p50": round(pct(lat, 50) * 1e6, 1), "p99": round(pct(lat, 99) * 1e6, 1),
                               "mean": round(statistics.mean(lat) * 1e6, 1), "n": n}
        lat = []
        for i in range(min(n, 1000)):
            body = json.dumps({"action": "work_generate", "hash": f"{i:064X}", "difficulty": "fffffff800000000"}).encode()
            t = time.perf_counter()
            req = urllib.request.Request(f"http://{srv.address}", data=body, method="POST")
            with urllib.request.urlopen(req, timeout=10) as r:
                json.loads(r.read())
            lat.append(time.perf_counter() - t)
        out["new_connection_us"] = {"p50": round(pct(lat, 50) * 1e6, 1), "p99": round(pct(lat, 99) * 1e6, 1),
                                    "n": len(lat)}
    finally:
        srv.stop()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
