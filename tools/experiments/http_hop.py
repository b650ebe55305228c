"""Round 5 probe: the HTTP hop with an instant stub engine (no GPU): raw-socket keep-alive RTT, bench's
KeepAliveClient RTT, and WorkServer.handle() called directly."""
import sys, time, json, statistics, socket, os
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "nano-dpow_amd")); sys.path.insert(0, ROOT)
from nanopow._lib import SearchResult, NPOW_OK
from nanopow.server import HttpWorkServer, WorkServer
class T:
    def wait(self, timeout=None): return SearchResult(NPOW_OK, 5, 0xffffffffffffffff, 1)
class E:
    def submit(self, root, thr, start=0, device_mask=0, cancel=None): return T()
    def work_value(self, r, n): return 0
ws = WorkServer(E(), max_active=64)
srv = HttpWorkServer(ws, "127.0.0.1", 0).start()
h, p = srv.address.split(":")
s = socket.create_connection((h, int(p))); s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
def raw(i):
    body = json.dumps({"action": "work_generate", "hash": f"{i + 1:064X}", "difficulty": "fffffe0000000000"}).encode()
    s.sendall(b"POST / HTTP/1.1\r\nHost: x\r\nContent-Type: application/json\r\nContent-Length: %d\r\n\r\n" % len(body) + body)
    buf = b""
    while b"\r\n\r\n" not in buf: buf += s.recv(65536)
    head, _, rest = buf.partition(b"\r\n\r\n")
    n = int([l.split(b":")[1] for l in head.split(b"\r\n") if l.lower().startswith(b"content-length")][0])
    while len(rest) < n: rest += s.recv(65536)
    return rest
def timeit(f, n=3000):
    for i in range(300): f(i)
    ts = []
    for i in range(n):
        t = time.perf_counter(); f(i); ts.append(time.perf_counter() - t)
    return round(statistics.median(ts) * 1e6, 1)
import bench
cli = bench.KeepAliveClient(srv.address)
out = {"raw_socket_rtt_us": timeit(raw),
       "bench_client_rtt_us": timeit(lambda i: cli.post({"action": "work_generate", "hash": f"{i + 1:064X}", "difficulty": "fffffe0000000000"})),
       "direct_handle_us": timeit(lambda i: ws.handle({"action": "work_generate", "hash": f"{i + 1:064X}", "difficulty": "fffffe0000000000"}))}
print(json.dumps(out))
srv.stop()
