"""Pin the oracle before trusting it (CPU only).

The oracle is two independent CPU restatements of the work value
(oracle/blake2b_oracle.c generic RFC 7693 BLAKE2b, and stdlib hashlib), checked
here against every committed golden vector: the 4096+ random triples, the
known answers (Nano genesis work; the reference's own docs/specification.md:30,45
example, which is *invalid* work), and the exhaustive sweep fixtures.
"""
import hashlib
import os

import pytest

import oracle
from conftest import load_golden

M64 = (1 << 64) - 1


def test_generic_blake2b_matches_hashlib():
    data = bytes(range(256)) * 3
    for n in [0, 1, 40, 127, 128, 129, 255, 256, 257, 700]:
        for outlen in [1, 8, 20, 32, 48, 64]:
            assert oracle.blake2b(data[:n], outlen) == hashlib.blake2b(data[:n], digest_size=outlen).digest()


def test_rfc7693_appendix_a_abc():
    # RFC 7693 Appendix A: BLAKE2b-512("abc")
    want = ("ba80a53f981c4d0d6a2797b69f12f6e94c212f14685ac4b74b12bb6fdbffa2d1"
            "7d87c5392aab792dc252d5de4533cc9518d38aa8dbf1925ab92386edd4009923")
    assert oracle.blake2b(b"abc", 64).hex() == want


def test_work_values_fixture_both_oracles():
    g = load_golden("work_values.json")
    roots = [bytes.fromhex(r) for r, _, _ in g["triples"]]
    nonces = [int(n, 16) for _, n, _ in g["triples"]]
    want = [int(v, 16) for _, _, v in g["triples"]]
    assert len(want) >= 4096
    assert oracle.work_values(roots, nonces) == want
    assert [oracle.work_value_hashlib(r, n) for r, n in zip(roots, nonces)] == want


def test_known_answers():
    g = load_golden("known_answers.json")
    for c in g["cases"]:
        root, nonce = bytes.fromhex(c["hash"]), int(c["work"], 16)
        v = oracle.work_value(root, nonce)
        assert f"{v:016x}" == c["value"]
        for thr, valid in c["valid"].items():
            assert (v >= int(thr, 16)) == valid
    genesis = g["cases"][0]
    assert genesis["value"] == "fffffff4000d3dac"
    spec_example = g["cases"][1]  # reference docs: a format illustration, not valid work
    assert spec_example["value"] == "1ce5be0f61328fc2"


def test_sweep_fixtures_hits_revalidate():
    g = load_golden("sweeps_small.json")
    for c in g["cases"]:
        root, thr = bytes.fromhex(c["root"]), int(c["threshold"], 16)
        for h in c["hits"]:
            assert oracle.work_value_hashlib(root, int(h, 16)) >= thr


@pytest.mark.parametrize("idx", [16, 17, 18])
def test_sweep_fixture_hashlib_ranges_c_oracle(idx):
    """The hashlib-exhaustive fixture ranges (incl. the one crossing 2^64 -> 0)
    re-derived by the C oracle: pins its completeness and wraparound."""
    c = load_golden("sweeps_small.json")["cases"][idx]
    assert c["method"].startswith("hashlib exhaustive")
    hits = oracle.sweep(bytes.fromhex(c["root"]), int(c["threshold"], 16), int(c["start"], 16), c["count"])
    assert [f"{h:016x}" for h in hits] == c["hits"]


def test_sweep_fixture_one_full_2p28_range_c_oracle():
    c = load_golden("sweeps_small.json")["cases"][0]
    assert c["count"] == 1 << 28
    hits = oracle.sweep(bytes.fromhex(c["root"]), int(c["threshold"], 16), 0, c["count"])
    assert [f"{h:016x}" for h in hits] == c["hits"]


def test_sweep_2p36_fixture_if_present():
    path = os.path.join(os.path.dirname(__file__), "golden", "sweep_2p36.json")
    if not os.path.exists(path):
        pytest.skip("sweep_2p36.json not generated yet")
    g = load_golden("sweep_2p36.json")
    root, thr = bytes.fromhex(g["root"]), int(g["threshold"], 16)
    hits = [int(h, 16) for h in g["hits"]]
    assert g["count"] == 1 << 36 and 60 < len(hits) < 220  # Poisson(128)
    assert hits == sorted(hits)
    for n in hits:
        assert oracle.work_value_hashlib(root, n) >= thr


def test_sweep_2p36_prefix_pinned_by_hashlib_2p30():
    """The 2^36 fixture (C oracle) below 2^30 equals the fffffff8 subset of a hashlib-only
    exhaustive scan of [0, 2^30) at fffff000."""
    g36 = load_golden("sweep_2p36.json")
    g30 = load_golden("sweep_2p30_hashlib.json")
    assert g30["root"] == g36["root"] and g30["start"] == "0000000000000000" and g30["count"] == 1 << 30
    root, send, low = bytes.fromhex(g30["root"]), int(g36["threshold"], 16), int(g30["threshold"], 16)
    hits30 = [int(h, 16) for h in g30["hits"]]
    assert 900 < len(hits30) < 1150 and hits30 == sorted(hits30)  # Poisson(1024)
    vals = {n: oracle.work_value_hashlib(root, n) for n in hits30}
    assert all(v >= low for v in vals.values())
    assert [n for n in hits30 if vals[n] >= send] == [int(h, 16) for h in g36["hits"] if int(h, 16) < 1 << 30]


def test_sweep_2p36_fixture_pinned_by_hashlib_in_full():
    """The whole 2^36 fixture equals a hashlib-only exhaustive scan of [0, 2^36)
    (tests/golden/gen_hashlib_2p36.py: the reference's own CPU path, 6 processes, 3.2 h in the
    build container): the C oracle that made sweep_2p36.json is pinned on every nonce of the range,
    not only on its hits."""
    g36 = load_golden("sweep_2p36.json")
    gh = load_golden("sweep_2p36_hashlib.json")
    assert gh["generator"] == "tests/golden/gen_hashlib_2p36.py" and gh["method"].startswith("hashlib.blake2b")
    for k in ("root", "threshold", "start", "count"):
        assert gh[k] == g36[k], k
    assert gh["hits"] == g36["hits"]
