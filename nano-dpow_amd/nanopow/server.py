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
Every reply a search produces was re-validated on the CPU inside libnanopow
before it reaches this layer.
"""
from __future__ import annotations

import json
import logging
import os
import random
import threading
import time
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from typing import Any, Dict, List, Optional, Protocol

from . import work as W
from ._lib import NPOW_CANCELLED, NPOW_OK, CancelToken, NanoPowError, SearchResult

log = logging.getLogger("nanopow.server")


class SearchTicket(Protocol):
    def wait(self, timeout: Optional[float] = None) -> Optional[SearchResult]: ...


class SearchEngine(Protocol):
    """What the server needs from an engine (libnanopow's :class:`nanopow.Engine`)."""

    def submit(self, root: bytes, threshold: int, start: int = 0, device_mask: int = 0,
               max_nonces_per_device: int = 0, cancel: Optional[CancelToken] = None) -> SearchTicket: ...

    def work_value(self, root: bytes, nonce: int) -> int: ...


class Job:
    __slots__ = ("root", "threshold", "cancel", "done", "reply", "active", "t_queued", "waiters", "t_started")

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

    def resolve(self, reply: Dict[str, Any]) -> None:
        if not self.done.is_set():
            self.reply = reply
            self.done.set()


class WorkServer:
    """Request dispatcher: a FIFO (or shuffled) queue in front of the engine's work pool."""

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
        self._dispatcher: Optional[threading.Thread] = None

    # -- lifecycle ---------------------------------------------------------------------
    def start(self) -> "WorkServer":
        with self._lock:
            if self._running:
                return self
            self._running = True
        self._dispatcher = threading.Thread(target=self._dispatch_loop, name="nanopow-dispatch", daemon=True)
        self._dispatcher.start()
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
        if self._dispatcher is not None:
            self._dispatcher.join(timeout=10)
        deadline = time.time() + 10
        with self._lock:
            while self._inflight and time.time() < deadline:
                self._lock.wait(0.1)

    # -- dispatch ----------------------------------------------------------------------
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
        job = self._enqueue(root, threshold)
        job.done.wait()
        return dict(job.reply)

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
            job = self._enqueue(self.rng.getrandbits(256).to_bytes(32, "little"), threshold)
            job.done.wait()
            if "work" not in job.reply:
                return {"error": "Benchmark failed", "hint": "Work generation failure"}
        ms = (time.perf_counter() - t0) * 1000.0
        return {"count": str(count), "difficulty": W.fmt_u64(threshold),
                "multiplier": W.fmt_multiplier(W.to_multiplier(threshold, self.base)),
                "duration": str(int(round(ms))), "average": str(int(round(ms / count))),
                "hint": "Times in milliseconds"}

    # -- queue + worker ----------------------------------------------------------------
    def _enqueue(self, root: bytes, threshold: int) -> Job:
        with self._lock:
            if not self._running:
                j = Job(root, threshold)
                j.resolve({"error": "Work generation failed (see logs for details)"})
                return j
            # the same root at the same threshold queued or running: share its result
            for j in self._inflight + self._queue:
                if j.root == root and j.threshold == threshold and not j.cancel.is_set:
                    j.waiters += 1
                    return j
            job = Job(root, threshold)
            self._queue.append(job)
            self._lock.notify_all()
            return job

    def _next_job(self) -> Optional[Job]:
        with self._lock:
            while self._running and (not self._queue or len(self._inflight) >= self.max_active):
                self._lock.wait()
            if not self._running:
                return None
            idx = self.rng.randrange(len(self._queue)) if self.shuffle else 0
            job = self._queue.pop(idx)
            job.active = True
            self._inflight.append(job)
            return job

    def _dispatch_loop(self) -> None:
        while True:
            job = self._next_job()
            if job is None:
                return
            job.t_started = time.perf_counter()
            try:
                ticket = self.engine.submit(job.root, job.threshold, start=self.rng.getrandbits(64),
                                            device_mask=self.device_mask, cancel=job.cancel)
            except Exception as e:  # never leave a client waiting
                log.error("Error computing work: %s", e)
                self._complete(job, {"error": "Work generation failed (see logs for details)"})
                continue
            threading.Thread(target=self._await, args=(job, ticket), name="nanopow-await", daemon=True).start()

    def _await(self, job: Job, ticket: SearchTicket) -> None:
        try:
            res = ticket.wait()
            if res is not None and res.status == NPOW_OK:
                reply = {"work": W.fmt_u64(res.nonce), "difficulty": W.fmt_u64(res.value),
                         "multiplier": W.fmt_multiplier(W.to_multiplier(res.value, self.base))}
                log.info("Generated for %s in %.0fms for difficulty %016x", job.root.hex().upper(),
                         (time.perf_counter() - job.t_started) * 1000.0, job.threshold)
            elif res is not None and res.status == NPOW_CANCELLED:
                reply = {"error": "Cancelled"}
            else:
                reply = {"error": "Work generation failed (see logs for details)"}
        except NanoPowError as e:
            log.error("Error computing work: %s", e)
            reply = {"error": "Work generation failed (see logs for details)"}
        except Exception as e:  # never leave a client waiting
            log.exception("work loop failure: %s", e)
            reply = {"error": "Work generation failed (see logs for details)"}
        self._complete(job, reply)

    def _complete(self, job: Job, reply: Dict[str, Any]) -> None:
        job.resolve(reply)
        with self._lock:
            if job in self._inflight:
                self._inflight.remove(job)
            self._lock.notify_all()


# ---------------------------------------------------------------------------------------
class _Handler(BaseHTTPRequestHandler):
    protocol_version = "HTTP/1.1"
    server_version = "nanopow-work-server/0.1"
    work_server: WorkServer  # set on the subclass

    def log_message(self, fmt: str, *args: Any) -> None:  # route to logging
        log.debug("%s - %s", self.address_string(), fmt % args)

    def _send(self, code: int, obj: Dict[str, Any]) -> None:
        body = json.dumps(obj).encode()
        self.send_response(code)
        self.send_header("Content-Type", "application/json")
        self.send_header("Content-Length", str(len(body)))
        self.end_headers()
        self.wfile.write(body)

    def do_POST(self) -> None:  # noqa: N802
        n = int(self.headers.get("Content-Length") or 0)
        raw = self.rfile.read(n) if n else b""
        try:
            req = json.loads(raw.decode("utf-8")) if raw else None
        except (UnicodeDecodeError, json.JSONDecodeError):
            req = None
        if req is None:
            self._send(200, {"error": "Failed to deserialize JSON"})
            return
        self._send(200, self.work_server.handle(req))

    def do_GET(self) -> None:  # noqa: N802
        self._send(405, {"error": "Can only POST requests"})


class _Listener(ThreadingHTTPServer):
    # socketserver's default listen backlog is 5: a burst of concurrent work_generate
    # connections (many clients, or one client's precache wave) would overflow it and wait
    # out TCP's 1-s SYN retry.
    request_queue_size = 1024


class HttpWorkServer:
    """WorkServer behind a threaded HTTP/1.1 listener (one thread per connection)."""

    def __init__(self, work_server: WorkServer, host: str = "127.0.0.1", port: int = 7000) -> None:
        handler = type("Handler", (_Handler,), {"work_server": work_server})
        self.work_server = work_server
        self.httpd = _Listener((host, port), handler)
        self.httpd.daemon_threads = True
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
