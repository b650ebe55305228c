"""Host logic: threshold / multiplier math and CLI parsing (CPU)."""
import pytest

from nanopow import work as W
from nanopow.__main__ import parse_args


def test_multiplier_roundtrip_dpow_formulas():
    # dpow_server.py:250-255 / 275-280: multiplier = (2^64-base)/(2^64-d), d = 2^64-(2^64-base)/m
    base = W.DEFAULT_BASE
    assert W.to_multiplier(base, base) == 1.0
    assert W.from_multiplier(1.0, base) == base
    assert W.to_multiplier(W.RECEIVE_THRESHOLD, base) == pytest.approx(1 / 64)
    assert W.from_multiplier(1 / 64, base) == W.RECEIVE_THRESHOLD
    assert W.from_multiplier(8.0, base) == 0xffffffff00000000
    for m in [0.5, 1.5, 2.0, 7.3]:
        assert W.to_multiplier(W.from_multiplier(m, base), base) == pytest.approx(m, rel=1e-9)


def test_threshold_parsing():
    assert W.parse_threshold("fffffff800000000") == W.SEND_THRESHOLD
    assert W.parse_threshold("FFFFFE0000000000") == W.RECEIVE_THRESHOLD
    assert W.parse_threshold("0") == 0
    for bad in ["", "g", "-1", "1" * 17, 5, "+f", "0x1f", " ff", "ff ", "f_f", "0X10"]:
        with pytest.raises(W.RequestError):
            W.parse_threshold(bad)


def test_requested_threshold_precedence():
    assert W.requested_threshold({}, 123) == 123
    assert W.requested_threshold({"multiplier": 1}, W.DEFAULT_BASE) == W.DEFAULT_BASE
    assert W.requested_threshold({"difficulty": "ff", "multiplier": 2}, W.DEFAULT_BASE) == 0xff


def test_work_and_hash_parsing():
    assert W.parse_hash({"hash": "AB" * 32}) == b"\xab" * 32
    assert W.parse_work({"work": "62f05417dd3fb691"}) == 0x62f05417dd3fb691
    assert W.parse_work({"work": "1"}) == 1
    assert W.parse_work({"work": "FFFFFFFFFFFFFFFF"}) == (1 << 64) - 1
    assert W.fmt_u64(1) == "0000000000000001"
    # int(x, 16) alone would take these (a negative work value would then be masked and validated)
    for bad in ["-1", "+f", "0x1f", " ff", "f_f", "ff\n", "１"]:
        with pytest.raises(W.RequestError) as e:
            W.parse_work({"work": bad})
        assert e.value.error == "Bad work"


def test_gpu_spec_and_cli():
    assert W.parse_gpu_spec("0:0") == (0, 0, 1048576)
    assert W.parse_gpu_spec("0:3:4194304") == (0, 3, 4194304)
    with pytest.raises(ValueError):
        W.parse_gpu_spec("0")
    a = parse_args(["--gpu", "0:0", "-l", "127.0.0.1:7000", "--shuffle", "--gpu-local-work-size", "64"])
    assert a.gpu == ["0:0"] and a.listen == "127.0.0.1:7000" and a.shuffle and a.local_work_size == 64
    assert parse_args([]).listen == "127.0.0.1:7000"


def test_cpu_threads_out_of_range_rejected():
    from nanopow.__main__ import main
    assert main(["--cpu-threads", "-1"]) == 2
    assert main(["--cpu-threads", "5000"]) == 2


def test_cli_with_cpu_threads_serves_the_transcript(monkeypatch):
    """`python -m nanopow --cpu-threads 2 --gpu 0:0 -l 127.0.0.1:P` starts (the reference's
    launch pattern, client/README.md:31, plus nano-work-server.exe @1681064 `cpu_threads`) and serves
    the WorkHandler transcript.  The engine is the oracle stand-in with 2 logical devices, the second
    playing the CPU workers' device: the CLI must ask the engine for 2 CPU threads and search over GPU 0
    and the CPU device (mask 0b11).  On the GPU the real CPU workers are tested in
    tests/test_gpu_pool.py::test_cpu_workers_beside_the_gpu."""
    import json
    import threading
    import urllib.request

    import oracle
    from conftest import load_golden
    from fake_engine import OracleEngine
    from nanopow import _lib
    from nanopow.__main__ import build, parse_args

    seen = {}

    def fake_engine(cpu_threads=0):
        seen["cpu_threads"] = cpu_threads
        e = OracleEngine(chunk=1 << 12, n_devices=2)
        e.cpu_device, e.gpu_mask = 1, 0b01
        return e
    monkeypatch.setattr(_lib, "engine", fake_engine)
    srv = build(parse_args(["--cpu-threads", "2", "--gpu", "0:0", "-l", "127.0.0.1:0", "--max-active", "1"]))
    assert not isinstance(srv, int)
    assert seen["cpu_threads"] == 2 and srv.work_server.device_mask == 0b11
    srv.start()
    try:
        def post(obj):
            req = urllib.request.Request(f"http://{srv.address}", data=json.dumps(obj).encode(), method="POST")
            with urllib.request.urlopen(req, timeout=30) as r:
                return json.loads(r.read())
        reqs = load_golden("workhandler_transcript.json")["requests"]
        assert post(reqs[0])["error"] == "Unknown command"
        g = dict(reqs[1], difficulty="fffff00000000000")
        r1 = post(g)
        assert oracle.work_value_hashlib(bytes.fromhex(g["hash"]), int(r1["work"], 16)) >= 0xfffff00000000000
        hold = dict(reqs[2], difficulty="ffffffffffffffff")
        box = {}
        th = threading.Thread(target=lambda: box.setdefault("r", post(hold)))
        th.start()
        import time
        time.sleep(0.3)
        assert post(reqs[3]) == {}
        th.join(10)
        assert box["r"] == {"error": "Cancelled"}
    finally:
        srv.stop()
    # a --gpu index past the GPUs (the CPU device is not a GPU) is refused
    assert build(parse_args(["--cpu-threads", "2", "--gpu", "0:1", "-l", "127.0.0.1:0"])) == 2


def test_gpu_threads_is_a_lower_bound_on_the_launch():
    """--gpu P:D:THREADS (nonces per launch in the reference, @1681064) raises the iteration cap
    only when a launch could not hold THREADS nonces."""
    from nanopow.__main__ import apply_threads

    class Stub:
        def __init__(self):
            self.tuning = None

        def stats(self, device):
            return type("S", (), {"grid": 1024, "pool_groups": 4})()  # 256 CUs x 4 workgroups of 512 lanes: 524,288 lanes

        def set_tuning(self, iters, poll, blocks):
            self.tuning = iters
    e = Stub()
    assert apply_threads(e, [(0, 0, 1048576)]) == 0 and e.tuning is None   # the default: 2 iterations' worth
    # a launch of cap c runs c / 2 wave iterations of 524,288 lanes: 2^32 nonces need 8,192 of them
    assert apply_threads(e, [(0, 0, 1 << 32)]) == 16384 and e.tuning == 16384
    assert apply_threads(e, [(0, 0, (1 << 32) + 1)]) == 16386
    assert apply_threads(e, [(0, 0, 1 << 31)]) == 0                       # exactly the default launch
    assert apply_threads(e, [(0, 0, 1 << 40)]) == 65536                   # capped


def test_sigterm_stops_the_server_like_ctrl_c():
    """`python -m nanopow` turns SIGTERM into the KeyboardInterrupt that ends serve_forever, so a stopped server exits
    normally and libnanopow's exit hook drains and frees the GPUs (tests/test_gpu_exit.py checks it on the GPU)."""
    import os
    import signal
    import time
    from nanopow.__main__ import _stop_on_sigterm
    old = signal.getsignal(signal.SIGTERM)
    try:
        _stop_on_sigterm()
        with pytest.raises(KeyboardInterrupt):
            os.kill(os.getpid(), signal.SIGTERM)
            time.sleep(2)
    finally:
        signal.signal(signal.SIGTERM, old)
