"""nano-work-server-compatible JSON work server on top of libnanopow.

Drop-in for the work server the DPoW client talks to
(client/README.md:31 ``nano-work-server --gpu 0:0 -l 127.0.0.1:7000``;
client/config_parse.py:18 default ``--worker_uri 127.0.0.1:7000``).  The
client's WorkHandler (client/work_handler.py) is the contract:

* ``start()`` POSTs ``{"action": "invalid"}`` with a 2 s timeout and reads
  ``['error']`` (work_handler.py:53) -> unknown actions answer
  ``{"error": "Unknown command", "hint": "Supported commands: ..."}``.
* ``loop()`` POSTs one ``work_generate {hash, difficulty}`` at a time and
  publishes ``res['work']`` (work_handler.py:104-117) -> the reply is
  ``{"work": "%016x", "difficulty": "%016x", "multiplier": "..."}``
  (nano-work-server.exe @1673856 field names).
* ``queue_cancel()`` POSTs ``work_cancel {hash}`` on a second connection while
  the generate is pending (work_handler.py:71-78) -> the pending generate
  returns ``{"error": "Cancelled"}`` and the cancel itself gets ``{}``.

Also served: ``work_validate`` (valid / valid_all / valid_receive / difficulty /
multiplier, @1680400..1680528), ``status`` (generating / queue_size,
@1679680) and ``benchmark`` (count -> duration / average / hint, @1679992..1680344).

Requests queue FIFO (``--shuffle``: random pick, nano-work-server.exe @1681064).
The reference serves one request at a time; here up to ``max_active`` queued
requests are handed to libnanopow's work pool at once (npow_submit), where
every selected GPU searches all of them in the same kernel launches, so a
burst of requests from many clients keeps the GPUs busy across request
boundaries.  ``max_active=1`` is the reference's strictly serial service.
Each connection's thread hands its own request to the engine and blocks there
for the result (no dispatcher or per-request threads).
Every reply a search produces was re-validated on the CPU inside libnanopow
before it reaches this layer.
"""
from __future__ import annotations

import json
import logging
import os
import queue
import random
import socket
import socketserver
import threading
import time
from typing import Any, Dict, List, Optional, Protocol

from . import work as W
from ._lib import NPOW_CANCELLED, NPOW_OK, CancelToken, NanoPowError, SearchResult

log = logging.getLogger("nanopow.server")

GENERATION_FAILED = {"error": "Work generation failed (see logs for details)"}


class SearchTicket(Protocol):
    def wait(self, timeout: Optional[float] = None) -> Optional[SearchResult]: ...


class SearchEngine(Protocol):
    """What the server needs from an engine (libnanopow's :class:`nanopow.Engine`)."""

    def submit(self, root: bytes, threshold: int, start: int = 0, device_mask: int = 0,
               max_nonces_per_device: int = 0, cancel: Optional[CancelToken] = None) -> SearchTicket: ...

    def work_value(self, root: bytes, nonce: int) -> int: ...


class Job:
    __slots__ = ("root", "threshold", "cancel", "done", "reply", "active", "t_queued", "waiters", "t_started",
                 "ticket", "dispatched", "collector")

    def __init__(self, root: bytes, threshold: int) -> None:
        self.root = root
        self.threshold = threshold
        self.cancel = CancelToken()
        self.done = threading.Event()
        self.reply: Dict[str, Any] = {}
        self.active = False
        self.t_queued = time.perf_counter()
        self.t_started = 0.0
        self.waiters = 1
        self.ticket: Optional[SearchTicket] = None
        self.dispatched = threading.Event()  # ticket set, or the job already resolved
        self.collector = False               # a request thread is collecting the ticket's result

    def resolve(self, reply: Dict[str, Any]) -> None:
        if not self.done.is_set():
            self.reply = reply
            self.done.set()
        self.dispatched.set()


class WorkServer:
    """Request dispatcher: a FIFO (or shuffled) queue in front of the engine's work pool.

    No thread of its own: a request is handed to the engine (npow_submit) by the request thread
    that queued it when fewer than max_active are in flight, otherwise by the request thread whose
    search ends next; each request thread then blocks in the engine (npow_wait, GIL released)
    for its own result.  A request costs no thread hand-off on the way in or out."""

    def __init__(self, engine: SearchEngine, base_threshold: int = W.DEFAULT_BASE, shuffle: bool = False,
                 device_mask: int = 0, rng: Optional[random.Random] = None, max_active: int = 4) -> None:
        if max_active < 1:
            raise ValueError("max_active must be >= 1")
        self.engine = engine
        self.base = base_threshold
        self.shuffle = shuffle
        self.device_mask = device_mask
        self.max_active = max_active
        self.rng = rng or random.Random(int.from_bytes(os.urandom(8), "little"))
        self._lock = threading.Condition()
        self._queue: List[Job] = []
        self._inflight: List[Job] = []
        self._running = False
        # tickets answered at their decision (npow_wait_result) and collected after the reply
        self._reap_q: "queue.SimpleQueue" = queue.SimpleQueue()
        self._reaper: Optional[threading.Thread] = None

    # -- lifecycle ---------------------------------------------------------------------
    def start(self) -> "WorkServer":
        with self._lock:
            self._running = True
        return self

    def stop(self) -> None:
        with self._lock:
            self._running = False
            pending = list(self._queue)
            self._queue.clear()
            for j in self._inflight:
                j.cancel.set()
            self._lock.notify_all()
        for j in pending:
            j.resolve({"error": "Cancelled"})
        deadline = time.time() + 10
        with self._lock:
            while self._inflight and time.time() < deadline:
                self._lock.wait(0.1)
            reaper, self._reaper = self._reaper, None
        if reaper is not None:
            self._reap_q.put(None)
            reaper.join(10)

    def _reap(self, ticket) -> None:
        """Collect a ticket whose reply has gone out (its other devices may still be stopping): one
        thread, started on first use, waits for each in turn (npow_wait)."""
        with self._lock:
            if self._reaper is None:
                self._reaper = threading.Thread(target=self._reap_loop, name="nanopow-reaper", daemon=True)
                self._reaper.start()
        self._reap_q.put(ticket)

    def _reap_loop(self) -> None:
        while True:
            t = self._reap_q.get()
            if t is None:
                return
            try:
                t.wait()
            except Exception as e:  # the reply is out; only log
                log.error("collecting a finished search: %s", e)

    # -- dispatch ----------------------------------------------------------------------
    def handle_body(self, raw: bytes) -> Dict[str, Any]:
        try:
            req = json.loads(raw.decode("utf-8")) if raw else None
        except (UnicodeDecodeError, json.JSONDecodeError):
            req = None
        if req is None:
            return {"error": "Failed to deserialize JSON"}
        return self.handle(req)

    def handle(self, req: Any) -> Dict[str, Any]:
        if not isinstance(req, dict):
            return {"error": "Failed to deserialize JSON"}
        action = req.get("action")
        try:
            if action == "work_generate":
                return self.work_generate(req)
            if action == "work_cancel":
                return self.work_cancel(req)
            if action == "work_validate":
                return self.work_validate(req)
            if action == "status":
                return self.status()
            if action == "benchmark":
                return self.benchmark(req)
            return {"error": "Unknown command", "hint": W.SUPPORTED}
        except W.RequestError as e:
            return e.reply()

    def work_generate(self, req: Dict[str, Any]) -> Dict[str, Any]:
        root = W.parse_hash(req)
        threshold = W.requested_threshold(req, self.base)
        return self._result(self._enqueue(root, threshold))

    def work_cancel(self, req: Dict[str, Any]) -> Dict[str, Any]:
        root = W.parse_hash(req)
        cancelled: List[Job] = []
        with self._lock:
            keep = []
            for j in self._queue:
                (cancelled if j.root == root else keep).append(j)
            self._queue[:] = keep
            for j in self._inflight:
                if j.root == root:
                    j.cancel.set()
        for j in cancelled:
            j.resolve({"error": "Cancelled"})
        log.info("Cancel %s", root.hex().upper())
        return {}

    def work_validate(self, req: Dict[str, Any]) -> Dict[str, Any]:
        root = W.parse_hash(req)
        nonce = W.parse_work(req)
        value = self.engine.work_value(root, nonce)
        out: Dict[str, Any] = {}
        if req.get("difficulty") is not None or req.get("multiplier") is not None:
            thr = W.requested_threshold(req, self.base)
            out["valid"] = "1" if value >= thr else "0"
        out["valid_all"] = "1" if value >= W.SEND_THRESHOLD else "0"
        out["valid_receive"] = "1" if value >= W.RECEIVE_THRESHOLD else "0"
        out["difficulty"] = W.fmt_u64(value)
        out["multiplier"] = W.fmt_multiplier(W.to_multiplier(value, self.base))
        return out

    def status(self) -> Dict[str, Any]:
        with self._lock:
            return {"generating": "1" if self._inflight else "0", "queue_size": str(len(self._queue))}

    def benchmark(self, req: Dict[str, Any]) -> Dict[str, Any]:
        count = W.parse_count(req)
        threshold = W.requested_threshold(req, self.base)
        log.info("Benchmarking %d samples at difficulty %016x (x%s)", count, threshold,
                 W.fmt_multiplier(W.to_multiplier(threshold, self.base)))
        t0 = time.perf_counter()
        for _ in range(count):
            reply = self._result(self._enqueue(self.rng.getrandbits(256).to_bytes(32, "little"), threshold))
            if "work" not in reply:
                return {"error": "Benchmark failed", "hint": "Work generation failure"}
        ms = (time.perf_counter() - t0) * 1000.0
        return {"count": str(count), "difficulty": W.fmt_u64(threshold),
                "multiplier": W.fmt_multiplier(W.to_multiplier(threshold, self.base)),
                "duration": str(int(round(ms))), "average": str(int(round(ms / count))),
                "hint": "Times in milliseconds"}

    # -- queue -------------------------------------------------------------------------
    def _enqueue(self, root: bytes, threshold: int) -> Job:
        with self._lock:
            if not self._running:
                j = Job(root, threshold)
                j.resolve(dict(GENERATION_FAILED))
                return j
            # the same root at the same threshold queued or running: share its result
            for j in self._inflight + self._queue:
                if j.root == root and j.threshold == threshold and not j.cancel.is_set:
                    j.waiters += 1
                    return j
            job = Job(root, threshold)
            self._queue.append(job)
            ready = self._pump_locked()
        self._submit(ready)
        return job

    def _pump_locked(self) -> List[Job]:
        """Move queued jobs in flight while fewer than max_active are (FIFO, or a random one
        with --shuffle); the caller submits them once the lock is released."""
        ready = []
        while self._running and self._queue and len(self._inflight) < self.max_active:
            idx = self.rng.randrange(len(self._queue)) if self.shuffle else 0
            job = self._queue.pop(idx)
            job.active = True
            job.t_started = time.perf_counter()
            self._inflight.append(job)
            ready.append(job)
        return ready

    def _submit(self, jobs: List[Job]) -> None:
        for job in jobs:
            try:
                job.ticket = self.engine.submit(job.root, job.threshold, start=self.rng.getrandbits(64),
                                                device_mask=self.device_mask, cancel=job.cancel)
            except Exception as e:  # never leave a client waiting
                log.error("Error computing work: %s", e)
                self._complete(job, dict(GENERATION_FAILED))
                continue
            job.dispatched.set()

    def _result(self, job: Job) -> Dict[str, Any]:
        """Block until the job's reply exists; the first request thread to get here after the
        job is in flight collects it from the engine, any other (a duplicate request) waits."""
        job.dispatched.wait()
        with self._lock:
            mine = not job.done.is_set() and job.ticket is not None and not job.collector
            if mine:
                job.collector = True
        if mine:
            self._complete(job, self._collect(job))
        job.done.wait()
        return dict(job.reply)

    def _collect(self, job: Job) -> Dict[str, Any]:
        try:
            t = job.ticket
            early = hasattr(t, "wait_result")
            # the reply as soon as the outcome is known (the reference answers when its result validates,
            # nano-work-server.exe @1669040), before a split search's other devices have stopped; the
            # ticket is collected after the reply (_reap)
            try:
                res = t.wait_result() if early else t.wait()
            finally:
                if early:  # collected even when the outcome is an error (else the engine keeps the job)
                    self._reap(t)
            if res is not None and res.status == NPOW_OK:
                log.info("Generated for %s in %.0fms for difficulty %016x", job.root.hex().upper(),
                         (time.perf_counter() - job.t_started) * 1000.0, job.threshold)
                return {"work": W.fmt_u64(res.nonce), "difficulty": W.fmt_u64(res.value),
                        "multiplier": W.fmt_multiplier(W.to_multiplier(res.value, self.base))}
            if res is not None and res.status == NPOW_CANCELLED:
                return {"error": "Cancelled"}
            return dict(GENERATION_FAILED)
        except NanoPowError as e:
            log.error("Error computing work: %s", e)
        except Exception as e:  # never leave a client waiting
            log.exception("work loop failure: %s", e)
        return dict(GENERATION_FAILED)

    def _complete(self, job: Job, reply: Dict[str, Any]) -> None:
        job.resolve(reply)
        with self._lock:
            if job in self._inflight:
                self._inflight.remove(job)
            ready = self._pump_locked()
            self._lock.notify_all()
        self._submit(ready)


# ---------------------------------------------------------------------------------------
_REASON = {200: "OK", 400: "Bad Request", 405: "Method Not Allowed", 413: "Payload Too Large"}
_MAX_LINE = 65536
_MAX_BODY = 1 << 20


class _Connection(socketserver.StreamRequestHandler):
    """One HTTP/1.1 client connection (keep-alive; the DPoW client's aiohttp session reuses it for
    every work_generate, client/work_handler.py:98-108): request line, headers, a JSON body ->
    one JSON reply written with ONE send (status line, headers and body together; TCP_NODELAY).
    A minimal parser: no email.parser header objects, no per-request allocation beyond the body."""
    disable_nagle_algorithm = True
    work_server: WorkServer  # set on the subclass

    def handle(self) -> None:
        rfile = self.rfile
        while True:
            line = rfile.readline(_MAX_LINE + 1)
            if not line:
                return
            if line in (b"\r\n", b"\n"):
                continue  # stray blank lines between requests (RFC 9112 2.2)
            parts = line.split()
            if len(parts) != 3 or not parts[2].startswith(b"HTTP/1."):
                self._send(400, {"error": "Bad request line"}, True)
                return
            method, version = parts[0], parts[2]
            close = version == b"HTTP/1.0"
            length, chunked = 0, False
            while True:
                h = rfile.readline(_MAX_LINE + 1)
                if h in (b"\r\n", b"\n", b""):
                    break
                name, _, value = h.partition(b":")
                name = name.strip().lower()
                if name == b"content-length":
                    try:
                        length = int(value.strip())
                    except ValueError:
                        length = -1
                elif name == b"connection":
                    v = value.strip().lower()
                    close = v == b"close" or (version == b"HTTP/1.0" and v != b"keep-alive")
                elif name == b"transfer-encoding":
                    chunked = b"chunked" in value.lower()
                elif name == b"expect" and value.strip().lower() == b"100-continue":
                    self.wfile.write(b"HTTP/1.1 100 Continue\r\n\r\n")
            if length < 0 or length > _MAX_BODY:
                self._send(413 if length > 0 else 400, {"error": "Bad Content-Length"}, True)
                return
            body = self._read_chunked() if chunked else (rfile.read(length) if length else b"")
            if body is None:
                self._send(400, {"error": "Bad chunked body"}, True)
                return
            if method == b"POST":
                self._send(200, self.work_server.handle_body(body), close)
            else:
                self._send(405, {"error": "Can only POST requests"}, close)
            if close:
                return

    def _read_chunked(self) -> Optional[bytes]:
        out = []
        total = 0
        while True:
            size_line = self.rfile.readline(_MAX_LINE + 1)
            try:
                n = int(size_line.split(b";")[0].strip(), 16)
            except ValueError:
                return None
            if n == 0:
                while self.rfile.readline(_MAX_LINE + 1) not in (b"\r\n", b"\n", b""):
                    pass  # trailers
                return b"".join(out)
            total += n
            if total > _MAX_BODY:
                return None
            out.append(self.rfile.read(n))
            self.rfile.readline(_MAX_LINE + 1)  # the chunk's CRLF

    def _send(self, code: int, obj: Dict[str, Any], close: bool) -> None:
        data = json.dumps(obj).encode()
        head = (f"HTTP/1.1 {code} {_REASON.get(code, 'OK')}\r\nContent-Type: application/json\r\n"
                f"Content-Length: {len(data)}\r\n{'Connection: close' + chr(13) + chr(10) if close else ''}\r\n")
        try:
            self.wfile.write(head.encode() + data)
        except OSError:
            pass  # the client went away; its request was answered as far as the server is concerned


class _Listener(socketserver.TCPServer):
    """Accepts connections and hands each to a connection thread (one per open connection: a DPoW
    client's keep-alive session holds its thread).  Threads that finish a connection wait for the
    next one (up to _MAX_IDLE of them) instead of exiting: a request on a new connection then costs
    a queue hand-off, not a thread start (round 5: ~0.3 ms per request on the MI355X box's host with
    a thread per connection, profiles/r05as_http_new_connection.json)."""
    # socketserver's default listen backlog is 5: a burst of concurrent work_generate
    # connections (many clients, or one client's precache wave) would overflow it and wait
    # out TCP's 1-s SYN retry, or be reset.  4,096 connections at once (BASELINE configs[3])
    # overflowed 1,024 with resets; the kernel caps this at net.core.somaxconn.
    request_queue_size = 8192
    allow_reuse_address = True
    _MAX_IDLE = 64

    def __init__(self, address, handler) -> None:
        super().__init__(address, handler)
        self._conns: "queue.SimpleQueue" = queue.SimpleQueue()
        self._pool_lock = threading.Lock()
        self._idle = 0       # connection threads waiting for a connection, not yet promised one
        self._closed = False

    def process_request(self, request, client_address) -> None:
        with self._pool_lock:
            spawn = self._idle == 0
            if not spawn:
                self._idle -= 1  # that thread takes this connection
        self._conns.put((request, client_address))
        if spawn:
            threading.Thread(target=self._connection_thread, name="nanopow-conn", daemon=True).start()

    def _connection_thread(self) -> None:
        while True:
            item = self._conns.get()
            if item is None:
                return
            request, client_address = item
            try:
                self.finish_request(request, client_address)
            except Exception:
                self.handle_error(request, client_address)
            finally:
                self.shutdown_request(request)
            with self._pool_lock:
                if self._closed or self._idle >= self._MAX_IDLE:
                    return
                self._idle += 1

    def server_close(self) -> None:
        super().server_close()
        with self._pool_lock:
            self._closed = True
            idle, self._idle = self._idle, 0
        for _ in range(idle):
            self._conns.put(None)


class HttpWorkServer:
    """WorkServer behind a threaded HTTP/1.1 listener (one thread per connection)."""

    def __init__(self, work_server: WorkServer, host: str = "127.0.0.1", port: int = 7000) -> None:
        handler = type("Connection", (_Connection,), {"work_server": work_server})
        self.work_server = work_server
        self.httpd = _Listener((host, port), handler)
        self._thread: Optional[threading.Thread] = None

    @property
    def address(self) -> str:
        h, p = self.httpd.server_address[:2]
        return f"{h}:{p}"

    def start(self) -> "HttpWorkServer":
        self.work_server.start()
        self._thread = threading.Thread(target=self.httpd.serve_forever, name="nanopow-http", daemon=True)
        self._thread.start()
        return self

    def serve_forever(self) -> None:
        self.work_server.start()
        self.httpd.serve_forever()

    def stop(self) -> None:
        self.work_server.stop()
        self.httpd.shutdown()
        self.httpd.server_close()
