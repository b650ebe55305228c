"""DPoW client side of the path: MQTT work/cancel messages -> work server -> result messages.

The reference's DPoW client (client/dpow_client.py) subscribes to ``work/<type>`` and
``cancel/<type>`` and feeds a WorkHandler (client/work_handler.py), which serialises the
requests to the work server over HTTP and publishes ``result/<type>``.  This module is the
same flow with the broker replaced by whatever delivers messages (a queue in the harness,
an MQTT client in deployment), so time-to-work can be measured from the message that asks
for work to the message that answers it -- the latency the DPoW server sees
(server/scripts/check_latency.py:18-39 times ``work`` -> ``result`` on the broker).

Message formats (dpow_client.py:38-39, 63-85):
  work/<type>    payload "<hash>,<difficulty>"           (hash: 64 hex chars)
  cancel/<type>  payload "<hash>"
  result/<type>  payload "<hash>,<work>,<payout account>"

WorkHandler semantics kept (work_handler.py:9-125): a request already queued or ongoing
for the same hash is ignored; the next request is picked at random from the queue
(WorkQueue._get); a cancel removes a queued hash, or, for an ongoing one, forgets it (the
result is then not published) and POSTs ``work_cancel``.  ``concurrency`` > 1 runs that many
request loops against the work server (the reference runs one).
"""
from __future__ import annotations

import asyncio
import json
import logging
import random
import time
import http.client
import threading
import urllib.parse
from typing import Awaitable, Callable, Dict, Optional, Tuple

log = logging.getLogger("nanopow.dpow")

WORK_TYPES = ("ondemand", "precache")


class MessageError(ValueError):
    pass


def parse_work_message(topic: str, payload: bytes) -> Tuple[str, str, str]:
    """``work/<type>`` + ``b"hash,difficulty"`` -> (work_type, hash, difficulty) (dpow_client.py:63-75)."""
    work_type = topic.split("/")[-1]
    try:
        block_hash, difficulty = payload.decode("utf-8").split(",")
    except (UnicodeDecodeError, ValueError) as e:
        raise MessageError(f"Could not parse message {topic}: {e}") from e
    if len(block_hash) != 64:
        raise MessageError(f"Invalid hash {block_hash}")
    return work_type, block_hash, difficulty


def parse_cancel_message(payload: bytes) -> str:
    """``cancel/<type>`` payload -> hash (dpow_client.py:77-85)."""
    try:
        block_hash = payload.decode("utf-8")
    except UnicodeDecodeError as e:
        raise MessageError(f"Could not parse cancel message: {e}") from e
    if len(block_hash) != 64:
        raise MessageError(f"Invalid hash {block_hash}")
    return block_hash


def result_message(work_type: str, block_hash: str, work: str, payout: str) -> Tuple[str, bytes]:
    """(topic, payload) of a result (dpow_client.py:38-39)."""
    return f"result/{work_type}", f"{block_hash},{work},{payout}".encode("utf-8")


class HttpWorker:
    """POSTs JSON actions to a work server over keep-alive HTTP/1.1 connections, as the
    WorkHandler's aiohttp session does (work_handler.py:51, :75-78, :104-108): each executor thread
    keeps one connection and reuses it; a request that finds its connection closed by the server
    is sent once more on a fresh one."""

    def __init__(self, uri: str, timeout: float = 300.0) -> None:
        self.uri = uri if uri.startswith("http") else f"http://{uri}"
        u = urllib.parse.urlsplit(self.uri)
        self.host, self.port = u.hostname or "127.0.0.1", u.port or 80
        self.path = u.path or "/"
        self.timeout = timeout
        self._local = threading.local()

    def _conn(self, fresh: bool = False) -> http.client.HTTPConnection:
        c = getattr(self._local, "conn", None)
        if c is None or fresh:
            if c is not None:
                c.close()
            c = self._local.conn = http.client.HTTPConnection(self.host, self.port, timeout=self.timeout)
        return c

    def _post(self, obj: Dict) -> Dict:
        body = json.dumps(obj)
        for attempt in (0, 1):
            c = self._conn(fresh=attempt == 1)
            try:
                c.request("POST", self.path, body, {"Content-Type": "application/json"})
                return json.loads(c.getresponse().read())
            except (http.client.RemoteDisconnected, ConnectionResetError, BrokenPipeError,
                    http.client.CannotSendRequest):
                if attempt == 1:
                    raise
        raise AssertionError("unreachable")

    async def post(self, obj: Dict) -> Dict:
        return await asyncio.get_running_loop().run_in_executor(None, self._post, obj)


PublishFn = Callable[[str, bytes], Awaitable[None]]


class DpowWorkHandler:
    """WorkHandler-equivalent: queue of requests -> work server -> published results."""

    def __init__(self, worker: HttpWorker, publish: PublishFn, payout: str, concurrency: int = 1,
                 rng: Optional[random.Random] = None) -> None:
        self.worker = worker
        self.publish = publish
        self.payout = payout
        self.concurrency = concurrency
        self.rng = rng or random.Random()
        self.queue: Dict[str, Tuple[str, str]] = {}   # hash -> (difficulty, work_type)
        self.ongoing: set = set()
        self._ready = asyncio.Event()
        self._tasks = []
        self.stats = {"queued": 0, "ignored": 0, "sent": 0, "cancelled": 0, "errors": 0}

    async def start(self) -> None:
        # WorkHandler.start: the probe must answer with an "error" field (work_handler.py:53)
        res = await self.worker.post({"action": "invalid"})
        if "error" not in res:
            raise RuntimeError(f"Worker not available at {self.worker.uri}")
        self._tasks = [asyncio.ensure_future(self._loop()) for _ in range(self.concurrency)]

    async def stop(self) -> None:
        for t in self._tasks:
            t.cancel()
        for t in self._tasks:
            try:
                await t
            except (asyncio.CancelledError, Exception):
                pass

    # -- message entry points (dpow_client.py handle_work / handle_cancel) --------------------
    async def on_message(self, topic: str, payload: bytes) -> None:
        try:
            if "cancel" in topic:
                await self.queue_cancel(parse_cancel_message(payload))
            elif "work" in topic:
                work_type, block_hash, difficulty = parse_work_message(topic, payload)
                await self.queue_work(work_type, block_hash, difficulty)
        except MessageError as e:
            log.warning("%s", e)

    async def queue_work(self, work_type: str, block_hash: str, difficulty: str) -> None:
        if block_hash in self.queue or block_hash in self.ongoing:
            self.stats["ignored"] += 1
            return
        self.queue[block_hash] = (difficulty, work_type)
        self.stats["queued"] += 1
        self._ready.set()

    async def queue_cancel(self, block_hash: str) -> None:
        if self.queue.pop(block_hash, None) is not None:
            self.stats["cancelled"] += 1
            return
        if block_hash in self.ongoing:
            self.ongoing.discard(block_hash)  # loop() will not publish it
            self.stats["cancelled"] += 1
            try:
                await self.worker.post({"action": "work_cancel", "hash": block_hash})
            except Exception as e:  # noqa: BLE001 -- logged like work_handler.py:79-80
                log.error("Work handler queue_cancel error: %s", e)

    async def _next(self) -> Tuple[str, str, str]:
        while not self.queue:
            self._ready.clear()
            await self._ready.wait()
        block_hash = self.rng.choice(list(self.queue))  # WorkQueue._get: random entry
        difficulty, work_type = self.queue.pop(block_hash)
        return block_hash, difficulty, work_type

    async def _loop(self) -> None:
        while True:
            block_hash, difficulty, work_type = await self._next()
            self.ongoing.add(block_hash)
            try:
                res = await self.worker.post({"action": "work_generate", "hash": block_hash,
                                              "difficulty": difficulty})
            except Exception as e:  # noqa: BLE001
                log.error("Work handler loop error: %s", e)
                self.ongoing.discard(block_hash)
                self.stats["errors"] += 1
                continue
            if block_hash not in self.ongoing:  # cancelled meanwhile
                continue
            self.ongoing.discard(block_hash)
            if "work" in res:
                await self.publish(*result_message(work_type, block_hash, res["work"], self.payout))
                self.stats["sent"] += 1
            elif res.get("error"):
                log.error("Unexpected reply from work server: %s", res["error"])


class LatencyProbe:
    """check_latency.py's bookkeeping: time from a ``work`` message to its ``result``."""

    def __init__(self) -> None:
        self.t_work: Dict[str, float] = {}
        self.latency: Dict[str, float] = {}
        self.results: Dict[str, Tuple[str, str]] = {}

    def saw_work(self, block_hash: str) -> None:
        self.t_work.setdefault(block_hash, time.perf_counter())

    def saw_result(self, topic: str, payload: bytes) -> None:
        block_hash, work, account = payload.decode("utf-8").split(",")
        if block_hash in self.t_work:
            self.latency[block_hash] = time.perf_counter() - self.t_work[block_hash]
        self.results[block_hash] = (work, account)


async def replay(handler: DpowWorkHandler, probe: LatencyProbe, schedule, drain_timeout: float = 60.0) -> float:
    """Deliver ``schedule`` = [(t_offset_s, topic, payload), ...] to ``handler`` at those times
    (the broker's role), recording work messages in ``probe``; then wait until every uncancelled
    hash has a result (or ``drain_timeout``).  Returns the wall time."""
    t0 = time.perf_counter()
    cancelled = set()
    wanted = set()
    for t_off, topic, payload in sorted(schedule, key=lambda x: x[0]):
        dt = t0 + t_off - time.perf_counter()
        if dt > 0:
            await asyncio.sleep(dt)
        try:
            if "cancel" in topic:
                cancelled.add(parse_cancel_message(payload))
            elif "work" in topic:
                h = parse_work_message(topic, payload)[1]
                probe.saw_work(h)
                wanted.add(h)
        except MessageError:
            pass  # the handler logs and drops it
        await handler.on_message(topic, payload)
    deadline = time.perf_counter() + drain_timeout
    while time.perf_counter() < deadline:
        pending = [h for h in wanted if h not in probe.results and h not in cancelled]
        if not pending and not handler.queue and not handler.ongoing:
            break
        await asyncio.sleep(0.002)
    return time.perf_counter() - t0
