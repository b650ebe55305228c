"""End to end on the GPU: the WorkHandler transcript against the work server backed by libnanopow."""
import json
import threading
import time
import urllib.request

import pytest

import oracle
from conftest import load_golden
from nanopow.server import HttpWorkServer, WorkServer

pytestmark = pytest.mark.gpu


def post(addr, obj, timeout=60):
    req = urllib.request.Request(f"http://{addr}", data=json.dumps(obj).encode(), method="POST",
                                 headers={"Content-Type": "application/json"})
    with urllib.request.urlopen(req, timeout=timeout) as r:
        return json.loads(r.read())


@pytest.fixture()
def gpu_server(gpu_engine):
    srv = HttpWorkServer(WorkServer(gpu_engine), "127.0.0.1", 0).start()
    yield srv
    srv.stop()


def test_transcript_on_gpu(gpu_server):
    t = load_golden("workhandler_transcript.json")
    reqs = t["requests"]
    assert "error" in post(gpu_server.address, reqs[0])
    r = post(gpu_server.address, reqs[1])
    root, thr = bytes.fromhex(reqs[1]["hash"]), int(reqs[1]["difficulty"], 16)
    assert oracle.work_value_hashlib(root, int(r["work"], 16)) == int(r["difficulty"], 16) >= thr
    hold = dict(reqs[2], difficulty="ffffffffffffffff")
    box = {}
    th = threading.Thread(target=lambda: box.setdefault("r", post(gpu_server.address, hold)))
    th.start()
    time.sleep(0.5)
    t0 = time.time()
    assert post(gpu_server.address, reqs[3]) == {}
    th.join(10)
    assert box["r"] == {"error": "Cancelled"}
    assert time.time() - t0 < 2.0


def test_send_difficulty_generate_and_validate(gpu_server):
    for i in range(5):
        h = f"{i + 1:064X}"
        r = post(gpu_server.address, {"action": "work_generate", "hash": h, "difficulty": "fffffff800000000"})
        v = oracle.work_value_hashlib(bytes.fromhex(h), int(r["work"], 16))
        assert v >= 0xfffffff800000000 and r["difficulty"] == f"{v:016x}"
        chk = post(gpu_server.address, {"action": "work_validate", "hash": h, "work": r["work"]})
        assert chk["valid_all"] == "1" and chk["valid_receive"] == "1"


def test_multiplier_requests_on_gpu(gpu_server):
    """A work_generate by multiplier (nano-work-server.exe @1680488 "multiplier"; the rule of dpow_server.py:250-305,
    restated in nanopow/work.py): the threshold derived from the base difficulty, the work re-validated under hashlib
    at it, and the reply's difficulty / multiplier those of the work's own value (SURVEY.md §8 A6 on the GPU path)."""
    from nanopow import work as W
    for i, m in enumerate(["1.0", "2.5", "0.125"]):
        h = f"{i + 100:064X}"
        thr = W.from_multiplier(float(m), W.DEFAULT_BASE)
        r = post(gpu_server.address, {"action": "work_generate", "hash": h, "multiplier": m})
        v = oracle.work_value_hashlib(bytes.fromhex(h), int(r["work"], 16))
        assert v >= thr and r["difficulty"] == f"{v:016x}", (m, r)
        assert float(r["multiplier"]) == pytest.approx(W.to_multiplier(v, W.DEFAULT_BASE), rel=1e-9), (m, r)


def test_benchmark_on_gpu(gpu_server):
    """`benchmark` (nano-work-server.exe @1679992..1680344): count searches of random roots at the
    base difficulty, timed end to end; fields and arithmetic as the reference reports them."""
    t = time.perf_counter()
    r = post(gpu_server.address, {"action": "benchmark", "count": 32})
    wall_ms = (time.perf_counter() - t) * 1e3
    assert set(r) == {"count", "difficulty", "multiplier", "duration", "average", "hint"}
    assert r["count"] == "32" and r["difficulty"] == "fffffff800000000" and float(r["multiplier"]) == 1.0
    assert r["hint"] == "Times in milliseconds"
    d, a = int(r["duration"]), int(r["average"])
    assert 0 < d <= wall_ms + 1 and abs(a - d / 32) <= 1
    # 32 searches at 2^29 expected nonces each on one MI355X (~27 Gnonce/s): ~20 ms apiece
    assert 2 <= a <= 200, r
    # at receive difficulty (2^23 expected nonces) every search is sub-millisecond on average
    r = post(gpu_server.address, {"action": "benchmark", "count": 50, "difficulty": "fffffe0000000000"})
    assert r["difficulty"] == "fffffe0000000000" and float(r["multiplier"]) == 1 / 64 and int(r["average"]) <= 5


def test_dpow_messages_to_results_on_gpu(gpu_engine):
    """MQTT-style work/cancel messages -> WorkHandler-equivalent (2 loops) -> HTTP work server ->
    libnanopow -> result messages; every result re-validates under hashlib, cancelled hashes
    publish nothing (client/dpow_client.py:38-39, 63-85; client/work_handler.py)."""
    import asyncio
    import random
    from nanopow import dpow
    srv = HttpWorkServer(WorkServer(gpu_engine, max_active=4), "127.0.0.1", 0).start()
    rng = random.Random(21)
    hashes = [bytes(rng.getrandbits(8) for _ in range(32)).hex().upper() for _ in range(24)]
    sched = [(0.002 * i, "work/ondemand", f"{h},fffffe0000000000".encode()) for i, h in enumerate(hashes)]
    never = [f"{0xEE00 + i:064X}" for i in range(3)]
    sched += [(0.01, "work/precache", f"{h},ffffffffffffffff".encode()) for h in never]
    sched += [(0.2, "cancel/precache", h.encode()) for h in never]
    published = []

    async def main():
        probe = dpow.LatencyProbe()

        async def publish(topic, payload):
            published.append((topic, payload))
            probe.saw_result(topic, payload)
        h = dpow.DpowWorkHandler(dpow.HttpWorker(srv.address, timeout=60), publish, "nano_test", concurrency=4)
        await h.start()
        wall = await dpow.replay(h, probe, sched, drain_timeout=60)
        await h.stop()
        return probe, wall
    try:
        probe, wall = asyncio.run(main())
    finally:
        srv.stop()
    assert wall < 30
    got = {}
    for topic, payload in published:
        bh, work, acct = payload.decode().split(",")
        assert topic == "result/ondemand" and acct == "nano_test"
        assert oracle.work_value_hashlib(bytes.fromhex(bh), int(work, 16)) >= 0xfffffe0000000000
        got[bh] = work
    assert set(got) == set(hashes)
    assert all(h not in probe.results for h in never)
