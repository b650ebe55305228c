#!/usr/bin/env python3
"""Pin BASELINE configs[2]'s fixture with the reference CPU path alone (build container only).

tests/golden/sweep_2p36.json (every valid nonce of [0, 2^36) for its root at fffffff800000000)
was produced by the C oracle, every hit then re-hashed by hashlib: hashlib confirmed each hit
but could not notice one the oracle missed.  This script scans the whole range with
hashlib.blake2b(digest_size=8) -- the CPU reference BASELINE.json names -- in one process per
core and writes tests/golden/sweep_2p36_hashlib.json: the complete hashlib hit list, which
tests/test_oracle.py requires to equal the fixture's.

Run: python3 tests/golden/gen_hashlib_2p36.py [processes]   (~2 h on 6 cores; resumable: progress
is kept in /tmp/nanopow_sweep_2p36_hashlib.progress.json)
"""
import hashlib
import json
import multiprocessing
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
PROGRESS = "/tmp/nanopow_sweep_2p36_hashlib.progress.json"
CHUNK = 1 << 26


def scan(job):
    """Every n in [lo, lo + CHUNK) with LE_u64(blake2b-64(LE64(n) || root)) >= threshold."""
    root, thr, lo = job
    b2 = hashlib.blake2b
    hits = []
    for n in range(lo, lo + CHUNK):
        d = b2(n.to_bytes(8, "little") + root, digest_size=8).digest()
        if d[7] == 255 and int.from_bytes(d, "little") >= thr:  # thr's top byte is 0xff
            hits.append(n)
    return lo, hits


def main() -> int:
    procs = int(sys.argv[1]) if len(sys.argv) > 1 else max(1, (os.cpu_count() or 2) - 2)
    fx = json.load(open(os.path.join(HERE, "sweep_2p36.json")))
    root, thr = bytes.fromhex(fx["root"]), int(fx["threshold"], 16)
    assert thr >> 56 == 0xff and int(fx["start"], 16) == 0
    count = fx["count"]
    done = {}
    if os.path.exists(PROGRESS):
        p = json.load(open(PROGRESS))
        if p.get("root") == fx["root"] and p.get("threshold") == fx["threshold"]:
            done = {int(k): v for k, v in p["chunks"].items()}
    todo = [lo for lo in range(0, count, CHUNK) if lo not in done]
    t0 = time.time()
    with multiprocessing.Pool(procs) as pool:
        for k, (lo, hits) in enumerate(pool.imap_unordered(scan, [(root, thr, lo) for lo in todo]), 1):
            done[lo] = [f"{h:016x}" for h in hits]
            if k % 8 == 0 or k == len(todo):
                with open(PROGRESS + ".tmp", "w") as f:
                    json.dump({"root": fx["root"], "threshold": fx["threshold"],
                               "chunks": {str(a): b for a, b in done.items()}}, f)
                os.replace(PROGRESS + ".tmp", PROGRESS)
                print(f"{len(done)}/{count // CHUNK} chunks, {time.time() - t0:.0f} s", flush=True)
    hits = sorted(int(h, 16) for v in done.values() for h in v)
    out = {"generator": "tests/golden/gen_hashlib_2p36.py", "root": fx["root"], "threshold": fx["threshold"],
           "start": fx["start"], "count": count,
           "method": f"hashlib.blake2b(digest_size=8) exhaustive over [0, 2^36) in {procs} processes "
                     f"(Python {sys.version.split()[0]})",
           "hits": [f"{h:016x}" for h in hits]}
    with open(os.path.join(HERE, "sweep_2p36_hashlib.json"), "w") as f:
        json.dump(out, f, indent=1)
        f.write("\n")
    same = out["hits"] == fx["hits"]
    print(f"{len(hits)} hits; equal to sweep_2p36.json: {same}")
    return 0 if same else 1


if __name__ == "__main__":
    sys.exit(main())
