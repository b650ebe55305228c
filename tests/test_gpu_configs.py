"""BASELINE.json configs[3] and configs[4] at full size on the GPU, on one MI355X exposed as 8
logical devices (NANOPOW_VIRTUAL_DEVICES=8: every request is split over 8 disjoint strides, each
logical device with its own stream and pool worker, as on an 8-GPU node).

configs[3] "DPoW burst: 4096 concurrent random block hashes batched across 8xMI355X with
mid-search MQTT-style work_cancel": 4,096 work_generate POSTs at fffffff800000000, all at once on
their own connections, to the JSON work server in a child process (tests/config_server.py); 25 %
of them get a work_cancel at a uniform time in [0, 0.5 x the expected burst time] -- the
reference client sends it on a second connection while the generate is pending
(client/work_handler.py:61-80) and reads no callback for it (:104-114).
configs[4] "Sustained node throughput at epoch-2 send difficulty with per-GPU nonce striding":
60 s of fresh roots through the work pool, 4 in flight per device (tests/config_sustained_worker.py).
"""
import http.client
import json
import os
import random
import subprocess
import sys
import threading
import time

import pytest

import oracle
from conftest import ROOT

pytestmark = pytest.mark.gpu

SEND = 0xfffffff800000000
N_BURST = 4096


def burst_root(i: int) -> bytes:
    import hashlib
    return hashlib.blake2b(b"config3-burst" + i.to_bytes(8, "little"), digest_size=32).digest()


def _post(address, obj, timeout=600):
    host, port = address.rsplit(":", 1)
    c = http.client.HTTPConnection(host, int(port), timeout=timeout)
    try:
        c.request("POST", "/", json.dumps(obj), {"Content-Type": "application/json"})
        return json.loads(c.getresponse().read())
    finally:
        c.close()


@pytest.mark.timeout(400)
def test_config3_burst_of_4096_with_cancels_over_8_devices():
    env = dict(os.environ, NANOPOW_VIRTUAL_DEVICES="8")
    p = subprocess.Popen([sys.executable, os.path.join(ROOT, "tests", "config_server.py")], env=env,
                         stdin=subprocess.PIPE, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    try:
        hello = json.loads(p.stdout.readline())
        addr = hello["address"]
        assert hello["devices"] == 8
        roots = [burst_root(i) for i in range(N_BURST)]
        rng = random.Random(2025)
        cancel_set = set(rng.sample(range(N_BURST), N_BURST // 4))
        expected_s = N_BURST * float(1 << 29) / 27e9
        cancel_at = sorted((rng.uniform(0.0, 0.5 * expected_s), i) for i in cancel_set)
        replies = [None] * N_BURST
        go = threading.Event()

        def client(i):
            go.wait()
            try:
                replies[i] = _post(addr, {"action": "work_generate", "hash": roots[i].hex().upper(),
                                          "difficulty": f"{SEND:016x}"})
            except Exception as e:  # recorded, asserted below
                replies[i] = {"exception": repr(e)}

        cancel_replies = []

        def canceller():
            go.wait()
            t0 = time.perf_counter()
            for t_c, i in cancel_at:
                time.sleep(max(0.0, t0 + t_c - time.perf_counter()))
                cancel_replies.append(_post(addr, {"action": "work_cancel", "hash": roots[i].hex().upper()}))

        ths = [threading.Thread(target=client, args=(i,), daemon=True) for i in range(N_BURST)]
        for t in ths:
            t.start()
        tc = threading.Thread(target=canceller, daemon=True)
        tc.start()
        t0 = time.perf_counter()
        go.set()
        for t in ths:
            t.join(360)
        wall = time.perf_counter() - t0
        tc.join(60)
        p.stdin.write("stats\n")
        p.stdin.flush()
        stats = json.loads(p.stdout.readline())
        assert p.wait(60) == 0
    finally:
        if p.poll() is None:
            p.kill()
    assert all(r is not None and "exception" not in r for r in replies), [r for r in replies if r and "exception" in r][:3]
    assert len(cancel_replies) == len(cancel_set) and all(r == {} for r in cancel_replies)
    won = [i for i in range(N_BURST) if "work" in replies[i]]
    for i in won:  # every reply with work re-validates under the reference CPU path
        v = oracle.work_value_hashlib(roots[i], int(replies[i]["work"], 16))
        assert v >= SEND and int(replies[i]["difficulty"], 16) == v, (i, replies[i])
    for i in range(N_BURST):
        if i not in cancel_set:
            assert "work" in replies[i], (i, replies[i])
        elif "work" not in replies[i]:
            assert replies[i] == {"error": "Cancelled"}, (i, replies[i])
    cancelled = sum(1 for i in cancel_set if "work" not in replies[i])
    assert cancelled > len(cancel_set) // 4  # most cancels land mid-search
    # accounting: the nonces every search reports (cancelled ones up to the cancel) are exactly what
    # the 8 devices' counters hashed; every device took part
    # every request reached the engine except those cancelled while still queued in the server
    assert N_BURST - cancelled <= stats["searches"] <= N_BURST
    assert stats["job_nonces"] == sum(stats["device_nonces"]), stats
    assert all(n > 0 for n in stats["launches"])
    gnps = stats["job_nonces"] / wall / 1e9
    print(json.dumps({"config": 3, "requests": N_BURST, "won": len(won), "cancelled": cancelled,
                      "engine_searches": stats["searches"], "wall_s": round(wall, 2), "gnps": round(gnps, 3)}))


@pytest.mark.timeout(300)
def test_config4_sustained_60s_over_8_devices():
    env = dict(os.environ, NANOPOW_VIRTUAL_DEVICES="8", SINGLE_S="8", SUSTAINED_S="60", DEPTH="4")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "config_sustained_worker.py")], env=env,
                       capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-4000:]
    out = json.loads(p.stdout.strip().splitlines()[-1])
    print(json.dumps(out))
    assert out["devices"] == 8 and out["invalid"] == 0
    assert out["sustained_s"] >= 60.0 and out["sustained_searches"] > 1000
    # striding every search over 8 devices with 32 in flight costs nothing against one at a time (measured 0.99-1.0;
    # recorded, and asserted only against the mechanism's failure: a device idle or hashing another's stride costs
    # at least one device's share, 1/8)
    assert out["ratio"] >= 1.0 - 1.0 / 8, out
