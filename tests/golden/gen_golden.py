#!/usr/bin/env python3
"""Generate the committed golden fixtures of tests/golden/ (run in the build container).

Every expected value here comes from Python's stdlib ``hashlib.blake2b``
(digest_size=8) -- the reference CPU path BASELINE.json names -- either
directly or, for exhaustive ranges too long for hashlib, from the C oracle
(oracle/blake2b_oracle.c) with EVERY reported hit re-hashed by hashlib and the
C oracle's completeness pinned by hashlib-exhaustive sub-ranges.

The reference repository itself holds no test vectors for this path (SURVEY.md
§4/§8c); the one hash/work pair in its docs (docs/specification.md:30,45) is
included as a known value (it is *invalid* work: value 0x1ce5be0f61328fc2).
The Nano live genesis work is an external known-answer test.

Synthetic roots follow SURVEY.md §8(d): R_i = blake2b(b"nanopow-bench" + LE64(i),
digest_size=32); the 2^36 sweep root is blake2b(b"nanopow-sweep", digest_size=32).

Usage:
  python3 tests/golden/gen_golden.py values      # work_values.json (4096 triples)
  python3 tests/golden/gen_golden.py kat         # known_answers.json
  python3 tests/golden/gen_golden.py sweeps      # sweeps_small.json  (~2 min on 8 cores)
  python3 tests/golden/gen_golden.py sweep36     # sweep_2p36.json    (~1 h on 8 cores)
"""
from __future__ import annotations

import hashlib
import json
import multiprocessing as mp
import os
import random
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
import oracle  # noqa: E402  (test infrastructure)

M64 = (1 << 64) - 1
SEND = 0xfffffff800000000      # epoch-2 send / change threshold
RECEIVE = 0xfffffe0000000000   # epoch-2 receive threshold
LOW = 0xfffff00000000000


def bench_root(i: int) -> bytes:
    return hashlib.blake2b(b"nanopow-bench" + i.to_bytes(8, "little"), digest_size=32).digest()


SWEEP_ROOT = hashlib.blake2b(b"nanopow-sweep", digest_size=32).digest()


def hl_value(root: bytes, nonce: int) -> int:
    return int.from_bytes(hashlib.blake2b((nonce & M64).to_bytes(8, "little") + root, digest_size=8).digest(),
                          "little")


def _hl_range(args):
    root, thr, start, count = args
    out = []
    for i in range(count):
        n = (start + i) & M64
        if hl_value(root, n) >= thr:
            out.append(n)
    return out


def hashlib_sweep(root: bytes, thr: int, start: int, count: int, procs: int = 8):
    """Exhaustive hashlib scan (multiprocessing, contiguous parts), hits in range order."""
    parts = []
    per = count // procs
    off = 0
    for p in range(procs):
        c = per + (count % procs if p == procs - 1 else 0)
        parts.append((root, thr, start + off, c))
        off += c
    with mp.Pool(procs) as pool:
        res = pool.map(_hl_range, parts)
    return [n for r in res for n in r]


def dump(name: str, obj) -> None:
    path = os.path.join(HERE, name)
    with open(path, "w") as f:
        json.dump(obj, f, indent=1)
        f.write("\n")
    print("wrote", path, os.path.getsize(path), "bytes")


def gen_values() -> None:
    rng = random.Random(0x4e414e4f)  # "NANO"
    triples = []
    for i in range(4096):
        root = bytes(rng.getrandbits(8) for _ in range(32))
        # a few structured nonces: 0, all-ones, carries across 32-bit halves
        if i < 8:
            nonce = [0, M64, 0xffffffff, 0x100000000, 0x00000000ffffffff ^ M64, 1, 1 << 63, 0x7fffffffffffffff][i]
        else:
            nonce = rng.getrandbits(64)
        triples.append([root.hex(), f"{nonce:016x}", f"{hl_value(root, nonce):016x}"])
    # structured roots
    for root in [bytes(32), b"\xff" * 32, bytes(range(32))]:
        for nonce in [0, 1, M64, 0x0123456789abcdef]:
            triples.append([root.hex(), f"{nonce:016x}", f"{hl_value(root, nonce):016x}"])
    dump("work_values.json", {
        "generator": "tests/golden/gen_golden.py values",
        "rule": "value = LE_u64(hashlib.blake2b(LE64(nonce) || root, digest_size=8)); columns: root hex, nonce %016x, value %016x",
        "triples": triples})


def gen_kat() -> None:
    genesis_root = "E89208DD038FBB269987689621D52292AE9C35941A7484756ECCED92A65093BA"
    genesis_work = "62f05417dd3fb691"
    spec_hash = "BFEB8AA91D346E6EFBB41D11FD247E48E0BC0DBC183DDEB9F26F3A98AA17522F"
    spec_work = "3108a2891093ce9e"
    cases = []
    for label, h, w, src in [
        ("nano live genesis open block (external KAT)", genesis_root, genesis_work, "external: Nano live genesis"),
        ("DPoW MQTT spec example (format illustration, not valid work)", spec_hash, spec_work,
         "reference docs/specification.md:30,45"),
    ]:
        v = hl_value(bytes.fromhex(h), int(w, 16))
        cases.append({"label": label, "source": src, "hash": h, "work": w, "value": f"{v:016x}",
                      "valid": {f"{t:016x}": v >= t for t in (0xffffffc000000000, SEND, RECEIVE, LOW)}})
    dump("known_answers.json", {"generator": "tests/golden/gen_golden.py kat", "cases": cases})


def gen_sweeps() -> None:
    t0 = time.time()
    cases = []
    # (1) 8 bench roots x [0, 2^28) at LOW and RECEIVE: C oracle, every hit re-hashed by hashlib
    for i in range(8):
        root = bench_root(i)
        hits = oracle.sweep(root, LOW, 0, 1 << 28)
        assert all(hl_value(root, n) >= LOW for n in hits)
        rec = [n for n in hits if hl_value(root, n) >= RECEIVE]
        cases.append({"root": root.hex(), "threshold": f"{LOW:016x}", "start": "0000000000000000",
                      "count": 1 << 28, "hits": [f"{n:016x}" for n in hits], "method": "c-oracle, hits re-hashed by hashlib"})
        cases.append({"root": root.hex(), "threshold": f"{RECEIVE:016x}", "start": "0000000000000000",
                      "count": 1 << 28, "hits": [f"{n:016x}" for n in rec],
                      "method": "subset of the fffff000 sweep, re-hashed by hashlib"})
        print(f"root {i}: {len(hits)} / {len(rec)} hits  t={time.time() - t0:.0f}s", flush=True)
    # (2) hashlib-exhaustive ranges: pin the C oracle's completeness (and the 2^64 wrap)
    for root, thr, start, count in [
        (bench_root(0), LOW, 0, 1 << 24),
        (bench_root(1), LOW, 0, 1 << 24),
        (bench_root(2), 0xffff000000000000, (M64 - (1 << 22)) + 1, 1 << 23),  # crosses 2^64 -> 0
    ]:
        hl = hashlib_sweep(root, thr, start, count)
        co = oracle.sweep(root, thr, start, count)
        assert hl == co, "C oracle disagrees with hashlib"
        cases.append({"root": root.hex(), "threshold": f"{thr:016x}", "start": f"{start:016x}", "count": count,
                      "hits": [f"{n:016x}" for n in hl], "method": "hashlib exhaustive (C oracle agrees)"})
        print(f"hashlib range {start:016x}+{count}: {len(hl)} hits  t={time.time() - t0:.0f}s", flush=True)
    dump("sweeps_small.json", {"generator": "tests/golden/gen_golden.py sweeps",
                               "rule": "every nonce in [start, start+count) mod 2^64 with value >= threshold, in range order",
                               "cases": cases})


def gen_sweep36() -> None:
    t0 = time.time()
    root = SWEEP_ROOT
    hits = oracle.sweep(root, SEND, 0, 1 << 36, threads=os.cpu_count() or 8)
    assert all(hl_value(root, n) >= SEND for n in hits), "hit failed hashlib re-validation"
    dt = time.time() - t0
    dump("sweep_2p36.json", {"generator": "tests/golden/gen_golden.py sweep36",
                             "root": root.hex(), "threshold": f"{SEND:016x}", "start": "0000000000000000",
                             "count": 1 << 36, "hits": [f"{n:016x}" for n in hits],
                             "method": f"c-oracle exhaustive on {os.cpu_count()} threads ({dt:.0f} s), every hit re-hashed by hashlib"})


def gen_sweep30() -> None:
    """the sweep root's [0, 2^30) scanned by hashlib alone (no C oracle in
    the loop) at fffff000 (~1,024 hits); its fffffff8 subset must equal the 2^36 fixture's prefix."""
    t0 = time.time()
    root, count = SWEEP_ROOT, 1 << 30
    hl = hashlib_sweep(root, LOW, 0, count, procs=os.cpu_count() or 8)
    co = oracle.sweep(root, LOW, 0, count)
    assert hl == co, "C oracle disagrees with hashlib"
    dt = time.time() - t0
    dump("sweep_2p30_hashlib.json", {"generator": "tests/golden/gen_golden.py sweep30",
                                     "root": root.hex(), "threshold": f"{LOW:016x}", "start": "0000000000000000",
                                     "count": count, "hits": [f"{n:016x}" for n in hl],
                                     "method": f"hashlib exhaustive on {os.cpu_count()} processes ({dt:.0f} s); "
                                               "C oracle agrees"})


if __name__ == "__main__":
    what = sys.argv[1:] or ["values", "kat", "sweeps"]
    for w in what:
        {"values": gen_values, "kat": gen_kat, "sweeps": gen_sweeps, "sweep36": gen_sweep36, "sweep30": gen_sweep30}[w]()
