"""The DPoW client side of the path (nanopow.dpow) on the CPU: MQTT-style work/cancel messages
through the WorkHandler-equivalent and the HTTP work server (oracle stand-in engine) to result
messages.  Message formats follow client/dpow_client.py:38-39, 63-85; queue / cancel semantics
client/work_handler.py:9-125."""
import asyncio
import random

import pytest

import oracle
from fake_engine import OracleEngine
from nanopow import dpow
from nanopow.server import HttpWorkServer, WorkServer

PAYOUT = "nano_1dpowtestpayoutaccount"


def test_message_formats():
    h = "AB" * 32
    assert dpow.parse_work_message("work/ondemand", f"{h},fffffff800000000".encode()) == \
        ("ondemand", h, "fffffff800000000")
    assert dpow.parse_cancel_message(h.encode()) == h
    assert dpow.result_message("precache", h, "0123456789abcdef", PAYOUT) == \
        ("result/precache", f"{h},0123456789abcdef,{PAYOUT}".encode())
    for bad in [b"abc,fff", b"no-comma", ("A" * 63 + ",ff").encode(), b"\xff\xfe,x"]:
        with pytest.raises(dpow.MessageError):
            dpow.parse_work_message("work/ondemand", bad)
    with pytest.raises(dpow.MessageError):
        dpow.parse_cancel_message(b"A" * 65)


def _run(schedule, concurrency=1, drain=30.0, engine=None):
    eng = engine or OracleEngine(chunk=1 << 12, delay=0.0005)
    srv = HttpWorkServer(WorkServer(eng, max_active=max(1, concurrency)), "127.0.0.1", 0).start()
    published = []

    async def main():
        probe = dpow.LatencyProbe()

        async def publish(topic, payload):
            published.append((topic, payload))
            probe.saw_result(topic, payload)

        h = dpow.DpowWorkHandler(dpow.HttpWorker(srv.address, timeout=60), publish, PAYOUT,
                                 concurrency=concurrency, rng=random.Random(1))
        await h.start()
        wall = await dpow.replay(h, probe, schedule, drain_timeout=drain)
        await h.stop()
        return h, probe, wall
    try:
        return asyncio.run(main()) + (published, eng)
    finally:
        srv.stop()


def test_replay_results_validate_and_cancels_publish_nothing():
    rng = random.Random(7)
    hashes = [bytes(rng.getrandbits(8) for _ in range(32)).hex().upper() for _ in range(6)]
    sched = [(0.001 * i, "work/ondemand" if i % 2 else "work/precache", f"{h},ffff000000000000".encode())
             for i, h in enumerate(hashes)]
    sched.append((0.0001, "work/ondemand", f"{hashes[0]},ffff000000000000".encode()))  # duplicate: ignored
    never = "CD" * 32
    sched.append((0.007, "work/ondemand", f"{never},ffffffffffffffff".encode()))       # never finishes ...
    sched.append((0.3, "cancel/ondemand", never.encode()))                             # ... cancelled
    sched.append((0.3, "work/ondemand", b"bad,message"))                               # logged, dropped
    h, probe, wall, published, eng = _run(sched)
    assert wall < 20, wall
    assert h.stats["ignored"] >= 1 and h.stats["cancelled"] == 1
    got = {}
    for topic, payload in published:
        bh, work, acct = payload.decode().split(",")
        assert acct == PAYOUT and len(work) == 16 and work == work.lower()
        assert topic == ("result/ondemand" if hashes.index(bh) % 2 else "result/precache")
        assert oracle.work_value_hashlib(bytes.fromhex(bh), int(work, 16)) >= 0xffff000000000000
        got[bh] = work
    assert set(got) == set(hashes) and never not in probe.results
    assert all(probe.latency[x] > 0 for x in hashes)


def test_concurrent_handler_loops():
    rng = random.Random(8)
    hashes = [bytes(rng.getrandbits(8) for _ in range(32)).hex() for _ in range(8)]
    sched = [(0.0, "work/ondemand", f"{x},ffff800000000000".encode()) for x in hashes]
    h, probe, wall, published, eng = _run(sched, concurrency=3)
    assert len(published) == 8 and h.stats["sent"] == 8
    for _, payload in published:
        bh, work, _ = payload.decode().split(",")
        assert oracle.work_value(bytes.fromhex(bh), int(work, 16)) >= 0xffff800000000000
