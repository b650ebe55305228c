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


def test_cpu_threads_rejected():
    from nanopow.__main__ import main
    assert main(["--cpu-threads", "4"]) == 2


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
