#!/usr/bin/env python3
"""bench.py -- Gnonce/s and time-to-work of the MI355X Nano PoW engine (libnanopow).

Workload = BASELINE.json configs[1] (the configuration its metric is quoted on):
"Send/change difficulty fffffff800000000 on one MI355X, single block hash,
p50/p99 time-to-work".  One step = one first-win search (the hot path behind a
``work_generate``: libnanopow npow_search through the C ABI) for a fresh
synthetic root R_i = blake2b(b"nanopow-bench" + LE64(i), 32) at threshold
fffffff800000000, from start nonce LE64(blake2b(b"start" + LE64(i), 8))
(SURVEY.md §8d).  Inputs are 32-byte roots; nothing is streamed from HBM.

value = Gnonce/s over the whole job = nonces hashed by all ranks (including
the rest of a chunk after each win) / max over ranks of the timed wall time.
p50 / p99 time-to-work are per-search wall times at the C ABI (rank 0 reports
the distribution over every rank's searches).

Multi-GPU (``torch.distributed.run``, one rank per GPU): every rank searches
its own roots on its own GPU (disjoint work, no data-path collective); gloo on
the CPU carries only the barrier and the max/sum of the timings.
Scaling is therefore "weak" (fixed searches per GPU).

roofline: the dominant kernel (npow_task_kernel<kSearch>) is int32-VALU bound.
achieved = nonces hashed in kernel x 2232 int32 ops/nonce /
kernel time, the kernel time measured by HIP events recorded on the stream the
kernel runs on (libnanopow stats); peak = 256 CUs x 128 int32 lanes/clk
(4 x SIMD-32) x 2.4 GHz = 78.6 Tops/s.
cpu_baseline (rank 0, N=1 only): the oracle's C restatement of the same work
value (oracle/blake2b_oracle.c, "port"), exhaustive scan of a bounded sample of
R_0's nonce space on the host cores; hashlib single-core rate alongside.
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import statistics
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
WORLD = int(os.environ.get("WORLD_SIZE", "1"))
LOCAL_RANK = int(os.environ.get("LOCAL_RANK", "0"))
if WORLD > 1 and "HIP_VISIBLE_DEVICES" not in os.environ:
    # one GPU per rank: the engine of rank r sees only GPU LOCAL_RANK (as device 0)
    os.environ["HIP_VISIBLE_DEVICES"] = str(LOCAL_RANK)
sys.path.insert(0, os.path.join(HERE, "nano-dpow_amd"))

SEND = 0xfffffff800000000
OPS_PER_NONCE = 2232                # int32 VALU ops of one 12-round compression
PEAK_TOPS = 256 * 128 * 2.4e9 / 1e12  # MI355X: 256 CU x (4 SIMD x 32 lanes) x 2.4 GHz = 78.6 Tops/s
METRIC = "Gnonce/s blake2b-64 per GPU & 8-GPU node; p50 time-to-work at fffffff8"


def bench_root(i: int) -> bytes:
    return hashlib.blake2b(b"nanopow-bench" + i.to_bytes(8, "little"), digest_size=32).digest()


def bench_start(i: int) -> int:
    return int.from_bytes(hashlib.blake2b(b"start" + i.to_bytes(8, "little"), digest_size=8).digest(), "little")


def pct(xs, p):
    xs = sorted(xs)
    if not xs:
        return None
    k = min(len(xs) - 1, max(0, int(round(p / 100.0 * (len(xs) - 1)))))
    return xs[k]


def cpu_baseline(seconds: float = 12.0):
    """Oracle C restatement on the host cores (bounded sample) + hashlib single-core rate."""
    sys.path.insert(0, os.path.join(HERE, "oracle"))
    import oracle  # test infrastructure: the CPU baseline leg only
    oracle.build()
    threads = min(16, os.cpu_count() or 1)  # the GPU box grants this process 16 CPUs
    root = bench_root(0)
    # calibrate on one thread, then size the sample for ~`seconds` on all threads
    t = time.perf_counter()
    oracle.sweep(root, SEND, 0, 1 << 20, threads=1)
    rate1 = (1 << 20) / (time.perf_counter() - t)
    count = int(rate1 * threads * seconds)
    t = time.perf_counter()
    hits = oracle.sweep(root, SEND, 1 << 40, count, threads=threads)
    dt = time.perf_counter() - t
    n = 200_000
    t = time.perf_counter()
    for i in range(n):
        hashlib.blake2b((i).to_bytes(8, "little") + root, digest_size=8).digest()
    hl = n / (time.perf_counter() - t)
    return {"value": round(count / dt / 1e9, 6), "unit": "Gnonce/s", "cores": threads, "kind": "port",
            "sample": f"oracle/blake2b_oracle.c exhaustive sweep of {count} nonces of R_0 from 2^40 at "
                      f"fffffff800000000 ({len(hits)} hits) on {threads} pthreads, {dt:.1f} s",
            "hashlib_1core_gnps": round(hl / 1e9, 6)}


def run_timed(search, stats, reset_stats, steps: int, warmup: int, rank: int, world: int, dist=None):
    """Warm up, then time exactly `steps` searches bracketed by barriers; reduce over ranks.

    search(i) -> (seconds, nonces_hashed); stats() -> (kernel_ms, kernel_nonces, launches).
    Returns the rank-0 view: (total_nonces, max_wall_s, all_ttw_s, kernel_ms, kernel_nonces, launches)
    with kernel_* summed over ranks."""
    base_idx = 1_000_000 * (rank + 1)
    for w in range(warmup):
        search(base_idx + 900_000 + w)
    reset_stats()
    if dist is not None:
        dist.barrier()
    # npow_search returns only after its streams drained, so the GPU is idle at both barriers
    t0 = time.perf_counter()
    ttw, nonces = [], 0
    for s in range(steps):
        dt, n = search(base_idx + s)
        ttw.append(dt)
        nonces += n
    if dist is not None:
        dist.barrier()
    wall = time.perf_counter() - t0
    kern_ms, kern_nonces, launches = stats()
    if dist is None:
        return nonces, wall, ttw, kern_ms, kern_nonces, launches
    import torch
    v = torch.tensor([float(nonces), float(kern_ms), float(kern_nonces), float(launches)], dtype=torch.float64)
    dist.all_reduce(v, op=dist.ReduceOp.SUM)
    w_t = torch.tensor([wall], dtype=torch.float64)
    dist.all_reduce(w_t, op=dist.ReduceOp.MAX)
    gathered = [None] * world
    dist.all_gather_object(gathered, ttw)
    all_ttw = [x for g in gathered for x in g]
    return int(v[0]), float(w_t[0]), all_ttw, float(v[1]), int(v[2]), int(v[3])


def result_line(world, steps, warmup, tot_nonces, max_wall, all_ttw, kern_ms, kern_nonces, launches):
    gnps = tot_nonces / max_wall / 1e9
    per_rank_kernel_s = kern_ms * 1e-3 / world
    achieved = (kern_nonces / world) * OPS_PER_NONCE / per_rank_kernel_s / 1e12 if kern_ms > 0 else 0.0
    return {
        "metric": METRIC,
        "value": round(gnps, 4),
        "unit": "Gnonce/s",
        "n_gpus": world,
        "steps": steps,
        "warmup": warmup,
        "ms_per_step": round(max_wall / steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u64",
        "data": "synthetic (random-looking 32-byte roots R_i = blake2b(b'nanopow-bench'+LE64(i)))",
        "config": {
            "workload": "BASELINE configs[1]: single block hash per search at send difficulty "
                        "fffffff800000000, first-win search, p50/p99 time-to-work",
            "threshold": "fffffff800000000",
            "searches_per_gpu": steps,
            "parallelism": f"dp{world} (disjoint roots per GPU, no collective)",
        },
        "p50_ttw_ms": round(pct(all_ttw, 50) * 1e3, 3),
        "p99_ttw_ms": round(pct(all_ttw, 99) * 1e3, 3),
        "mean_ttw_ms": round(statistics.mean(all_ttw) * 1e3, 3),
        "gnps_per_gpu": round(gnps / world, 4),
        "roofline": {
            "bound": "valu",
            "kernel": "npow_task_kernel<Mode::kSearch>",
            "achieved": round(achieved, 3),
            "peak": round(PEAK_TOPS, 3),
            "unit": "Tops/s (int32 VALU)",
            "frac": round(achieved / PEAK_TOPS, 4),
            "traffic": None,
            "ops_per_nonce": OPS_PER_NONCE,
            "kernel_gnps": round(kern_nonces / (kern_ms * 1e-3) / 1e9, 4) if kern_ms > 0 else None,
            "avg_launch_ms": round(kern_ms / launches, 4) if launches else None,
            "launches": launches,
        },
        "cpu_baseline": None,
    }


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=300, help="searches per rank in the timed region")
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--iters", type=int, default=0, help="override wave iterations per launch")
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", "0"))
    dist = None
    if WORLD > 1:
        import torch.distributed as dist  # gloo: barrier + scalar reductions only
        dist.init_process_group("gloo")

    import nanopow
    from nanopow import _lib
    eng = nanopow.engine()  # fails loudly without libnanopow.so / a GPU: no CPU fallback
    if args.iters:
        eng.set_tuning(args.iters, 0, 0)
    dev = 0

    def search(i):
        t = time.perf_counter()
        r = eng.search(bench_root(i), SEND, start=bench_start(i), device_mask=1 << dev)
        dt = time.perf_counter() - t
        if r.status != _lib.NPOW_OK:
            raise RuntimeError(f"search {i} returned status {r.status}")
        return dt, r.nonces_done

    def stats():
        st = eng.stats(dev)
        return st.kernel_ms, st.nonces, st.launches

    res = run_timed(search, stats, lambda: eng.reset_stats(dev), args.steps, args.warmup, rank, WORLD, dist)
    if rank == 0:
        line = result_line(WORLD, args.steps, args.warmup, *res)
        if WORLD == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline()
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
