#!/usr/bin/env python3
"""Capture the DPoW client's work-server request sequence (build container only).

Drives the reference caller, client/work_handler.py (WorkHandler.start /
queue_work / queue_cancel / loop, work_handler.py:50-125), against a recording
HTTP server and writes tests/golden/workhandler_transcript.json: the exact
JSON bodies it POSTs, in order, plus the replies given and the callbacks it
made.  Only that JSON is committed; the reference code does not travel.
tests/test_server.py replays the transcript against nanopow's server and
checks the replies satisfy what WorkHandler reads from them.

Run: python3 tests/golden/gen_transcript.py   (needs /root/reference and aiohttp)

``--live`` drives the same reference caller against THIS repository's work server instead of
a recorder: nanopow.server.HttpWorkServer backed by the oracle stand-in engine
(tests/fake_engine.py), through start() (the blocking `requests` probe), queue_work x N on the
aiohttp keep-alive session, a duplicate queue_work, queue_cancel of a queued hash (popped
locally, never sent) and of an in-flight hash (work_cancel on a second connection).  It writes
tests/golden/workhandler_live.json: every request and reply in server order with the
connection each came on, and every callback the client made.  tests/test_server.py checks it.
"""
from __future__ import annotations

import asyncio
import hashlib
import importlib.util
import json
import os
import sys
import threading
import time
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer

sys.dont_write_bytecode = True  # the reference tree is read-only
HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference/client/work_handler.py"
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
import oracle  # noqa: E402

H1 = hashlib.blake2b(b"transcript-1", digest_size=32).hexdigest().upper()
H2 = hashlib.blake2b(b"transcript-2", digest_size=32).hexdigest().upper()
DIFF = "fffff00000000000"

log = []
cancelled = set()
cond = threading.Condition()


class Rec(BaseHTTPRequestHandler):
    protocol_version = "HTTP/1.1"

    def log_message(self, *a):
        pass

    def do_POST(self):
        body = json.loads(self.rfile.read(int(self.headers["Content-Length"])))
        entry = {"t": round(time.monotonic(), 3), "request": body}
        with cond:
            log.append(entry)
        action = body.get("action")
        if action == "work_generate":
            h = body["hash"]
            if h == H2:  # hold it until cancelled
                with cond:
                    cond.wait_for(lambda: h in cancelled, timeout=10)
                reply = {"error": "Cancelled"}
            else:
                root = bytes.fromhex(h)
                _, nonce = oracle.search(root, int(body["difficulty"], 16), 0, 1 << 30)
                value = oracle.work_value(root, nonce)
                reply = {"work": f"{nonce:016x}", "difficulty": f"{value:016x}", "multiplier": "1.0"}
        elif action == "work_cancel":
            with cond:
                cancelled.add(body["hash"])
                cond.notify_all()
            reply = {}
        else:
            reply = {"error": "Unknown command",
                     "hint": "Supported commands: work_generate, work_cancel, work_validate, benchmark, status"}
        entry["reply"] = reply
        data = json.dumps(reply).encode()
        self.send_response(200)
        self.send_header("Content-Type", "application/json")
        self.send_header("Content-Length", str(len(data)))
        self.end_headers()
        self.wfile.write(data)


def drive_live(mod) -> dict:
    """The reference WorkHandler against nanopow's HttpWorkServer (oracle stand-in engine)."""
    sys.path.insert(0, os.path.join(HERE, ".."))
    sys.path.insert(0, os.path.join(HERE, "..", "..", "nano-dpow_amd"))
    from fake_engine import OracleEngine
    from nanopow.server import HttpWorkServer, WorkServer

    rec, conns = [], {}
    rec_lock = threading.Lock()
    peer = threading.local()  # the client (port) of the connection this request thread serves

    class RecordingWorkServer(WorkServer):
        def handle(self, req):
            with rec_lock:
                conn = conns.setdefault(peer.port, len(conns))
                entry = {"conn": conn, "request": req}
                rec.append(entry)
            reply = super().handle(req)
            with rec_lock:
                entry["reply"] = reply
            return reply

    srv = HttpWorkServer(RecordingWorkServer(OracleEngine(chunk=1 << 14), max_active=1), "127.0.0.1", 0)
    conn_cls = srv.httpd.RequestHandlerClass

    class PeerConnection(conn_cls):
        def handle(self):
            peer.port = self.client_address[1]
            super().handle()
    srv.httpd.RequestHandlerClass = PeerConnection
    srv.start()
    hashes = [hashlib.blake2b(b"live-%d" % i, digest_size=32).hexdigest().upper() for i in range(8)]
    hold = hashlib.blake2b(b"live-hold", digest_size=32).hexdigest().upper()
    queued = hashlib.blake2b(b"live-queued", digest_size=32).hexdigest().upper()
    callbacks, errors = [], []

    async def cb(client, work_type, block_hash, work):
        callbacks.append({"work_type": work_type, "hash": block_hash, "work": work})

    async def err_cb():
        errors.append(True)

    def requested(h):
        with rec_lock:
            return any(e["request"].get("hash") == h and e["request"].get("action") == "work_generate" for e in rec)

    async def drive():
        wh = mod.WorkHandler(srv.address, None, cb, err_cb)
        await wh.start()                                   # blocking requests probe (own connection)
        task = asyncio.ensure_future(wh.loop())
        await wh.queue_work("precache", hold, "ffffffffffffffff")   # never completes on its own
        for _ in range(200):
            if requested(hold):
                break
            await asyncio.sleep(0.02)
        await wh.queue_work("precache", hold, "ffffffffffffffff")   # duplicate of in-flight work: ignored
        await wh.queue_work("ondemand", queued, DIFF)               # queued behind it in the client ...
        await wh.queue_cancel(queued)                               # ... and cancelled there: never sent
        await wh.queue_cancel(hold)                                 # in flight: work_cancel, 2nd connection
        for i, h in enumerate(hashes):
            await wh.queue_work("ondemand" if i % 2 == 0 else "precache", h, DIFF)
        for _ in range(1000):
            if len(callbacks) >= len(hashes):
                break
            await asyncio.sleep(0.02)
        task.cancel()
        await wh.stop()

    try:
        asyncio.new_event_loop().run_until_complete(drive())
    finally:
        srv.stop()
    return {
        "generator": "tests/golden/gen_transcript.py --live (reference client/work_handler.py driven against "
                     "nanopow.server.HttpWorkServer with the oracle stand-in engine)",
        "difficulty": DIFF, "hashes": hashes, "hold": hold, "queued_then_cancelled": queued,
        "log": rec, "callbacks": callbacks, "error_callbacks": len(errors),
        "notes": "conn = the client connection (source port, numbered in order of appearance) a request arrived on: the probe is a blocking `requests` "
                 "POST (work_handler.py:53); work_generate / work_cancel go through the aiohttp session "
                 "(:75-78, :104-108), which reuses a connection once a reply has been read (:115) and opens "
                 "another while one is busy or left unread (the cancelled generate's reply is never read, :109-114).",
    }


def main() -> int:
    spec = importlib.util.spec_from_file_location("ref_work_handler", REF)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    if "--live" in sys.argv[1:]:
        out = drive_live(mod)
        path = os.path.join(HERE, "workhandler_live.json")
        with open(path, "w") as f:
            json.dump(out, f, indent=1)
            f.write("\n")
        print(json.dumps({k: out[k] for k in ("callbacks", "error_callbacks")}, indent=1))
        print(f"{len(out['log'])} requests -> {path}")
        return 0

    httpd = ThreadingHTTPServer(("127.0.0.1", 0), Rec)
    httpd.daemon_threads = True
    threading.Thread(target=httpd.serve_forever, daemon=True).start()
    uri = f"127.0.0.1:{httpd.server_address[1]}"
    callbacks = []

    async def cb(client, work_type, block_hash, work):
        callbacks.append({"work_type": work_type, "hash": block_hash, "work": work})

    async def err_cb():
        callbacks.append({"error_callback": True})

    async def drive():
        wh = mod.WorkHandler(uri, None, cb, err_cb)
        await wh.start()
        task = asyncio.ensure_future(wh.loop())
        await wh.queue_work("ondemand", H1, DIFF)
        for _ in range(200):
            if callbacks:
                break
            await asyncio.sleep(0.05)
        await wh.queue_work("precache", H2, DIFF)
        await asyncio.sleep(0.5)           # H2 is now in flight
        await wh.queue_cancel(H2)          # -> work_cancel on a second connection
        await asyncio.sleep(0.5)
        task.cancel()
        await wh.stop()

    asyncio.new_event_loop().run_until_complete(drive())
    httpd.shutdown()
    out = {
        "generator": "tests/golden/gen_transcript.py (reference client/work_handler.py driven against a recorder)",
        "requests": [e["request"] for e in log],
        "replies": [e.get("reply") for e in log],
        "callbacks": callbacks,
        "notes": "WorkHandler reads reply['error'] of the probe (work_handler.py:53), reply['work'] of a generate "
                 "(:116-117) and ignores the work_cancel reply (:75-78); a cancelled generate makes no callback (:109-114).",
    }
    path = os.path.join(HERE, "workhandler_transcript.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
        f.write("\n")
    print(json.dumps(out, indent=1))
    return 0


if __name__ == "__main__":
    sys.exit(main())
