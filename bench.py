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
p50_ttw_ms / max_ttw_ms describe the timed searches; after the timed region
rank 0 times --latency-searches (default 1,000) more searches on R_0..R_999 at
the C ABI for a real p50 / p99 of time-to-work (ttw_c_abi_ms), and 100
work_generate requests over one keep-alive HTTP connection (http_ttw_ms).

Multi-GPU, two ways (``--gpus N``):
  * under ``torch.distributed.run`` (WORLD_SIZE = N, the driver's scaling runs): one rank per GPU,
    every rank searching its own roots on its own GPU (disjoint work, no data-path collective);
    gloo on the CPU carries only the barrier and the max/sum of the timings.  A rank that already
    sees exactly one device (a launcher narrowed HIP_/CUDA_/ROCR_VISIBLE_DEVICES) keeps it; otherwise
    it takes the LOCAL_RANK-th visible device.  Afterwards every rank searches the same roots on
    disjoint strides, the first win cancelling the others through a shared word (node_ttw_ms);
  * in one process (WORLD_SIZE unset, N > 1): the product's own multi-GPU path -- the work pool
    over device_mask = N devices, N searches in flight, each split into N disjoint strides with
    first-found cancellation across the GPUs (npow_pool.cpp); afterwards one root at a time over
    all N (node_ttw_ms, with each search's overshoot: how long the other GPUs kept hashing after the
    host accepted the winner).  Fails if fewer than N devices are visible.
Scaling is "weak" either way (K searches per GPU).

roofline: the dominant kernel (npow_pool_kernel_ls2_arg<false>) is int32-VALU bound.
achieved = nonces hashed in kernel x 2232 int32 ops/nonce /
kernel time, the kernel time measured by HIP events recorded on the stream the
kernel runs on (libnanopow stats); peak = 256 CUs x 128 int32 lanes/clk
(4 x SIMD-32) x 2.4 GHz = 78.6 Tops/s.  frac_at_measured_sclk prices the same
achieved rate against 256 x 128 x the in-kernel shader clock of the timed
launches (s_memtime / s_memrealtime spans of one wave per XCD per launch,
libnanopow stats clock_mhz).
cpu_baseline (rank 0, N=1 only, run before the GPU is opened): the reference's
CPU path, hashlib.blake2b(digest_size=8), on every granted host core
(multiprocessing, disjoint ranges of R_0 from 2^40 at fffffff8, "reference");
the oracle's C restatement on the same cores and hashlib on one core alongside,
and the hashlib hit set checked against the C oracle's over the same range.

Other BASELINE.json configurations (``--workload``; not the driver's default line):
  allgpus   one process, every visible GPU on ONE root at a time (first win across
            GPUs, disjoint strides): p50/p99 time-to-work at N GPUs (config 2 at N>1);
  sweep     config 3: every hit of [0, 2^36) for the fixture root, ranks split the range,
            hit set compared with tests/golden/sweep_2p36.json (exact);
  burst     config 4: --roots requests at fffffff8 submitted at once to the work pool
            (npow_submit), 25 % cancelled at uniform times in [0, 0.5 x the expected
            burst time); every reply re-validated on the CPU (libnanopow npow_work_value);
  sustained config 5: --duration seconds of back-to-back fresh roots, --depth in flight.
  receive   config 1: single work_generate requests at receive difficulty fffffe0000000000,
            on the GPU (C ABI and HTTP server) next to the reference's CPU path
            (hashlib.blake2b, one core, and the oracle's C port on the host cores);
  regime    the 8-GPU time regime: one root at a time at ffffffc0 (2^26 nonces, ~1.9 ms on
            one GPU) over --gpus devices of the process, the next root submitted at the previous result;
            time-to-work against ln2 * 2^26 / kernel rate, node rate against kernel rate, the per-search
            fixed cost decomposed (node_ttw_8x_regime);
  dpow      the MQTT path end to end: --roots work messages at
            fffffff8 arriving as a Poisson stream at --rate per second, 25 % cancelled by
            a cancel message, delivered to the WorkHandler-equivalent (nanopow.dpow,
            --concurrency loops) -> HTTP work server -> engine -> result messages;
            p50/p99 = work message -> result message (server/scripts/check_latency.py).
"""
from __future__ import annotations

import argparse
import ctypes
import glob
import hashlib
import json
import os
import statistics
import sys
import threading
import time

HERE = os.path.dirname(os.path.abspath(__file__))
WORLD = int(os.environ.get("WORLD_SIZE", "1"))
LOCAL_RANK = int(os.environ.get("LOCAL_RANK", "0"))


def _ids(v):
    return [x.strip() for x in v.split(",") if x.strip()]


def rank_visibility(env, local_rank: int):
    """One GPU per rank under torch.distributed.run: the environment change (or None) that leaves
    the rank exactly one visible device, or raises SystemExit if it cannot.  HIP enumerates the
    devices ROCR_VISIBLE_DEVICES exposes, then applies HIP_VISIBLE_DEVICES (or, if that is unset,
    CUDA_VISIBLE_DEVICES) as indices into them.  A rank that already sees exactly one device -- a
    launcher narrowed one of the lists for it -- keeps it; a list of several is indexed by
    LOCAL_RANK; with none set the rank takes device LOCAL_RANK."""
    def get(k):  # an empty list is what a GPU-less container exports: as if unset
        v = env.get(k)
        return v if v is not None and v.strip() else None
    hip, cuda, rocr = get("HIP_VISIBLE_DEVICES"), get("CUDA_VISIBLE_DEVICES"), get("ROCR_VISIBLE_DEVICES")
    lst = hip if hip is not None else cuda
    if lst is not None:
        ids = _ids(lst)
        if len(ids) == 1:
            return None
        if local_rank >= len(ids):
            raise SystemExit(f"bench.py: LOCAL_RANK {local_rank} but only {len(ids)} visible devices "
                             f"({'HIP' if hip is not None else 'CUDA'}_VISIBLE_DEVICES={lst!r})")
        return {"HIP_VISIBLE_DEVICES": ids[local_rank]}
    if rocr is not None:
        ids = _ids(rocr)
        if len(ids) == 1:
            return None
        if local_rank >= len(ids):
            raise SystemExit(f"bench.py: LOCAL_RANK {local_rank} but ROCR_VISIBLE_DEVICES={rocr!r}")
    return {"HIP_VISIBLE_DEVICES": str(local_rank)}


if WORLD > 1:
    os.environ.update(rank_visibility(os.environ, LOCAL_RANK) or {})
sys.path.insert(0, os.path.join(HERE, "nano-dpow_amd"))

SEND = 0xfffffff800000000
OPS_PER_NONCE = 2232                # int32 VALU ops of one 12-round compression
PEAK_TOPS = 256 * 128 * 2.4e9 / 1e12  # MI355X: 256 CU x (4 SIMD x 32 lanes) x 2.4 GHz = 78.6 Tops/s
STREAM_INC = os.path.join(HERE, "nano-dpow_amd", "csrc", "npow_hash_asm_lockstep_ld.inc")


def stream_mix(path=STREAM_INC):
    """The shipped stream's instruction mix, from the generator's header line of the committed file:
    {opcode: count per nonce}, its VALU total, and the int32 ops it executes per nonce
    (v_lshl_add_u64 = one 64-bit add = 2 ops; xor, alignbit, shift 1 each; v_mov 0)."""
    import re
    with open(path) as f:
        head = f.read(2000)
    m = re.search(r"Per nonce: (\d+) VALU instructions \(([^)]*)\)", head)
    mix = {k: int(v) for k, v in (x.strip().rsplit(" ", 1) for x in m.group(2).split(","))}
    ops = sum(2 * c if op == "v_lshl_add_u64" else (0 if op.startswith("v_mov") else c) for op, c in mix.items())
    return {"valu": int(m.group(1)), "mix": mix, "executed_int32_ops": ops}


STREAM = {"kernel": "npow_pool_kernel_ls2_arg<false>", "sweep_kernel": "npow_sweep_kernel_ls2"}
# The issue model of the shipped stream (round 3, tools/experiments/dual_issue.py): a SIMD issues one
# half-rate instruction (v_alignbit_b32, v_lshl_add_u64) per quad-cycle, or two full-rate ones, and a
# full-rate instruction of another wave can ride in an alignbit's shadow (not in a 64-bit add's).  The
# quad-cycles of one 64-nonce wave-hash are then at least adds + alignbits + max(0, full - alignbits) / 2.
def issue_bound_cycles(mix):
    adds, aligns = mix["mix"].get("v_lshl_add_u64", 0), mix["mix"].get("v_alignbit_b32", 0)
    full = mix["valu"] - adds - aligns
    return 4 * (adds + aligns + max(0, full - aligns) / 2)
# rocprofv3 PMC passes of the bench's own command (tools/pmc_bench.sh), newest first
PMC_POOL = ("r06q_pmc_pool.json", "r06g_pmc_pool.json", "r06f_pmc_pool.json", "r05av_pmc_pool.json", "r05au_pmc_pool.json", "r05am_pmc_pool.json", "r05ak_pmc_pool.json", "r05f_pmc_pool.json", "r04j_pmc_pool.json", "r04i_pmc_pool.json", "r04h_pmc_pool.json", "r04g_pmc_pool.json", "r04f_pmc_pool.json", "r04e_pmc_pool.json", "r03s_pmc_pool.json", "r03w_pmc_pool.json", "r03p_pmc_pool.json", "r03_pmc_pool.json", "r02_ls2_pmc_pool.json")
PMC_SWEEP = ("r06q_pmc_sweep.json", "r06g_pmc_sweep.json", "r06f_pmc_sweep.json", "r05av_pmc_sweep.json", "r05au_pmc_sweep.json", "r05am_pmc_sweep.json", "r05ak_pmc_sweep.json", "r05f_pmc_sweep.json", "r04j_pmc_sweep.json", "r04i_pmc_sweep.json", "r04h_pmc_sweep.json", "r04g_pmc_sweep.json", "r04f_pmc_sweep.json", "r04e_pmc_sweep.json", "r03s_pmc_sweep.json", "r03w_pmc_sweep.json", "r03p_pmc_sweep.json", "r03_pmc_sweep.json", "r02_ls2_pmc_sweep.json")
METRIC = "Gnonce/s blake2b-64 per GPU & 8-GPU node; p50 time-to-work at fffffff8"
CSRC = os.path.join(HERE, "nano-dpow_amd", "csrc")


def build_sha16() -> str:
    """Identity of the libnanopow build: sha256 over the library's sources (kernel, generated streams,
    host engine, C ABI header, Makefile), file names included.  The same sources rebuild the same
    library, so a profile made from a bench line with this id describes this build."""
    h = hashlib.sha256()
    files = sorted(glob.glob(os.path.join(CSRC, "*.hip")) + glob.glob(os.path.join(CSRC, "*.cpp")) +
                   glob.glob(os.path.join(CSRC, "*.h")) + glob.glob(os.path.join(CSRC, "*.inc")) +
                   [os.path.join(CSRC, "Makefile"), os.path.join(HERE, "include", "nanopow.h")])
    for f in files:
        h.update(os.path.basename(f).encode() + b"\0")
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def timed_region_profile(build: str):
    """The committed rocprofv3 timed-region summary (tools/rocprof_timed_region.py) for this build: the
    newest profiles/*_rocprofv3_timed_region.txt whose build_sha16 line equals `build`, else the newest one
    at all (matches_this_build false).  Its fields as a dict, or None when there is none."""
    import re
    files = sorted(glob.glob(os.path.join(HERE, "profiles", "*_rocprofv3_timed_region.txt")), key=os.path.getmtime,
                   reverse=True)
    parsed = []
    for f in files:
        txt = open(f).read()
        m = re.search(r"^build_sha16 ([0-9a-f]{16})", txt, re.M)
        avg = re.search(r"timed region = the last (\d+) dispatches.*?average ([0-9.]+) ms", txt)
        npl = re.search(r"^nonces_per_launch ([0-9]+)", txt, re.M)
        fr = re.search(r"^frac_executed_from_profile ([0-9.]+)", txt, re.M)
        cy = re.search(r"^cycles_per_hash_from_profile ([0-9.]+)", txt, re.M)
        mz = re.search(r"^in_kernel_mhz ([0-9.]+)", txt, re.M)
        if not (m and avg and npl):
            continue
        parsed.append({"file": "profiles/" + os.path.basename(f), "build_sha16": m.group(1),
                       "matches_this_build": m.group(1) == build, "timed_dispatches": int(avg.group(1)),
                       "avg_dispatch_ms": float(avg.group(2)), "nonces_per_launch": int(npl.group(1)),
                       "frac_from_profile": float(fr.group(1)) if fr else None,
                       "in_kernel_mhz": float(mz.group(1)) if mz else None,
                       "cycles_per_hash_from_profile": float(cy.group(1)) if cy else None})
    for p in parsed:
        if p["matches_this_build"]:
            return p
    return parsed[0] if parsed else None


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


CHECK_THR = 0xfffff00000000000  # cpu_baseline: hits kept at this lower threshold for the parity cross-check


def search_to_result(eng, root: bytes, thr: int, start: int, mask: int):
    """One search as the work server serves it (round 4): submit, the outcome at the decision
    (npow_wait_result -- what the client is answered with), then the ticket collected (npow_wait_info:
    every device stopped, nonces_done complete).  Returns (seconds to the result, seconds to the
    collection, info).  Time-to-work is the first."""
    t = time.perf_counter()
    tk = eng.submit(root, thr, start=start, device_mask=mask)
    r = tk.wait_result()
    t_res = time.perf_counter() - t
    if r is None or r.status != 0:
        raise RuntimeError(f"search returned status {None if r is None else r.status}")
    info = tk.wait_info()
    return t_res, time.perf_counter() - t, info


def _hashlib_scan(job):
    """The reference CPU path (hashlib.blake2b(digest_size=8), dpow_server.py:130 rule value >= d)
    over nonces [start, start + count) of one root; returns (hits >= CHECK_THR, seconds)."""
    root, start, count = job
    b2 = hashlib.blake2b
    hits = []
    t = time.perf_counter()
    for n in range(start, start + count):
        if int.from_bytes(b2(n.to_bytes(8, "little") + root, digest_size=8).digest(), "little") >= CHECK_THR:
            hits.append(n)
    return hits, time.perf_counter() - t


def granted_cores() -> int:
    """Host cores this process may use: its affinity set, at most 16 (the GPU box grants a one-GPU
    job 16 CPUs; os.cpu_count() there shows the whole machine)."""
    try:
        n = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        n = os.cpu_count() or 1
    return max(1, min(16, n))


def cpu_baseline(seconds: float = 10.0):
    """The reference's CPU path on every granted host core: hashlib.blake2b(digest_size=8) in one
    process per core over disjoint ranges of R_0 from 2^40 (a bounded exhaustive sample, ~`seconds`
    of wall time).  Alongside: hashlib on one core, and the oracle's C restatement on the same cores
    over the same range, whose hit set must equal hashlib's.  Runs before the GPU is opened (fork)."""
    import multiprocessing
    sys.path.insert(0, os.path.join(HERE, "oracle"))
    import oracle  # test infrastructure: the CPU baseline leg only
    oracle.build()
    cores = granted_cores()
    root = bench_root(0)
    _, dt1 = _hashlib_scan((root, 0, 200_000))
    rate1 = 200_000 / dt1
    per = int(rate1 * seconds)
    base = 1 << 40
    with multiprocessing.get_context("fork").Pool(cores) as pool:
        t = time.perf_counter()
        parts = pool.map(_hashlib_scan, [(root, base + i * per, per) for i in range(cores)], chunksize=1)
        wall = time.perf_counter() - t
    total = cores * per
    hl_hits = sorted(h for hits, _ in parts for h in hits)
    t = time.perf_counter()
    c_hits = oracle.sweep(root, CHECK_THR, base, total, threads=cores)
    c_dt = time.perf_counter() - t
    n_send = sum(1 for h in hl_hits if oracle.work_value(root, h) >= SEND)
    return {"value": round(total / wall / 1e9, 6), "unit": "Gnonce/s", "cores": cores, "kind": "reference",
            "sample": f"hashlib.blake2b(digest_size=8) in {cores} processes (one per granted host core), exhaustive "
                      f"scan of {total} nonces of R_0 from 2^40 at fffffff800000000 ({n_send} hits; {len(hl_hits)} at "
                      f"fffff00000000000), {wall:.1f} s",
            "hashlib_1core_gnps": round(rate1 / 1e9, 6),
            "port_gnps": round(total / c_dt / 1e9, 6),
            "port": f"oracle/blake2b_oracle.c on {cores} pthreads over the same range, {c_dt:.1f} s",
            "hits_equal_port": hl_hits == c_hits}


class NodeQueue:
    """The timed searches of a multi-rank run as ONE node-wide queue: a counter in a file that every
    rank of this node draws from under flock (~10 us a draw).  A first-win search hashes a random
    number of nonces (exponential, coefficient of variation 1), so K fixed roots per rank would leave
    the ranks with the luckier roots idle at the closing barrier -- with K = 300 the slowest of 8
    ranks runs ~8 % past the mean.  Drawing from one queue, as a DPoW node's GPUs serve one request
    stream, every GPU stays busy until the N*K searches are done; ranks finish within about one
    search of each other."""

    @staticmethod
    def create(dist, rank: int, total: int):
        """The queue, or None on every rank if any rank cannot use the file (the ranks then fall
        back to K fixed roots each): every rank runs the same collectives either way."""
        import tempfile
        import torch
        box = [None]
        if rank == 0:
            try:
                fd, path = tempfile.mkstemp(prefix="nanopow_bench_queue_")
                os.write(fd, (0).to_bytes(8, "little"))
                os.close(fd)
                box = [path]
            except OSError:
                box = [None]
        dist.broadcast_object_list(box, src=0)
        q = None
        if box[0] is not None:
            try:
                q = NodeQueue(box[0], rank, total)
            except OSError:
                q = None
        ok = torch.tensor([1 if q is not None else 0], dtype=torch.int32)
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
        if int(ok[0]) == 1:
            return q
        if q is not None:
            q.close()
        elif rank == 0 and box[0] is not None:
            os.unlink(box[0])
        return None

    def __init__(self, path: str, rank: int, total: int):
        self.path, self.total, self.rank = path, total, rank
        self.fd = os.open(self.path, os.O_RDWR)

    def draw(self):
        import fcntl
        fcntl.flock(self.fd, fcntl.LOCK_EX)
        try:
            i = int.from_bytes(os.pread(self.fd, 8, 0), "little")
            if i < self.total:
                os.pwrite(self.fd, (i + 1).to_bytes(8, "little"), 0)
        finally:
            fcntl.flock(self.fd, fcntl.LOCK_UN)
        return i if i < self.total else None

    def close(self):
        try:
            os.close(self.fd)
            if self.rank == 0:
                os.unlink(self.path)
        except OSError:
            pass


class SharedWords:
    """32-bit words in a file every rank of this node maps (mmap, MAP_SHARED): cancel words of
    searches that all ranks run on ONE root.  The rank whose search wins raises the word; the
    other ranks' engines poll it as that search's cancel word (nanopow.CancelToken duck type:
    .address / .set()) and stop within microseconds.  Every rank runs the same collectives
    whatever happens locally (a rank without the mapping searches without a cancel word)."""

    class Word:
        def __init__(self, cw):
            self._w = cw

        @property
        def address(self) -> int:
            import ctypes
            return ctypes.addressof(self._w)

        def set(self) -> None:
            self._w.value = 1

        @property
        def is_set(self) -> bool:
            return bool(self._w.value)

    def __init__(self, dist, rank: int, n: int):
        import ctypes
        import mmap
        import tempfile
        box = [None]
        if rank == 0:
            try:
                fd, path = tempfile.mkstemp(prefix="nanopow_bench_cancel_")
                os.ftruncate(fd, 4 * n)
                os.close(fd)
                box = [path]
            except OSError:
                box = [None]
        dist.broadcast_object_list(box, src=0)
        self.path, self.rank, self.words, self.mm, self.f = box[0], rank, None, None, None
        if self.path is not None:
            try:
                self.f = open(self.path, "r+b")
                self.mm = mmap.mmap(self.f.fileno(), 4 * n)
                self.words = [ctypes.c_uint32.from_buffer(self.mm, 4 * i) for i in range(n)]
            except (OSError, ValueError):
                self.words = None

    def word(self, i: int):
        return SharedWords.Word(self.words[i]) if self.words is not None else None

    def close(self) -> None:
        # The mapping itself stays until the process exits: an engine must never poll a cancel
        # word whose page is gone, and the mmap cannot close while ctypes words point into it.
        self.words = None
        if self.f is not None:
            self.f.close()
        if self.rank == 0 and self.path is not None:
            try:
                os.unlink(self.path)
            except OSError:
                pass


def node_time_to_work(eng, dev: int, rank: int, world: int, dist, m: int, thr: int = SEND):
    """One root at a time searched by ALL ranks (north_star: the nonce space split into disjoint
    per-GPU strides, first found cancels the others): rank r scans start + r * 2^64/N; the
    winner raises the root's shared cancel word.  Runs after the timed region; returns (rank 0)
    {p50, p99, n, ...} of the winners' search times, or None on other ranks."""
    spacing = (1 << 64) // world
    words = SharedWords(dist, rank, m)
    recs = []
    try:
        for i in range(m):
            dist.barrier()
            tok = words.word(i)
            idx = 3_000_000 + i
            t = time.perf_counter()
            try:
                tk = eng.submit(bench_root(idx), thr, start=(bench_start(idx) + rank * spacing) & ((1 << 64) - 1),
                                device_mask=1 << dev, cancel=tok)
                r = tk.wait_result()  # the outcome at the decision: the winner raises the word at once
                dt = time.perf_counter() - t
                if r.status == 0 and tok is not None:
                    tok.set()
                recs.append((dt, r.status, tk.wait().nonces_done))
            except Exception:  # keep the collectives aligned; reported as a failed search
                recs.append((None, -1, 0))
        dist.barrier()
    finally:
        words.close()
    gathered = [None] * world
    dist.all_gather_object(gathered, recs)
    if rank != 0:
        return None
    ttw, failed, nonces, busy = [], 0, 0, 0.0
    cancelled = sum(1 for g in gathered for rec in g if rec[1] == 1)
    for i in range(m):
        wins = [g[i][0] for g in gathered if g[i][1] == 0]
        nonces += sum(g[i][2] for g in gathered)
        # the root occupies the node until its last rank returns (the winner, or a rank that saw
        # the winner's cancel word): the node's search time for that root
        busy += max((g[i][0] for g in gathered if g[i][0] is not None), default=0.0)
        if wins:
            ttw.append(min(wins))
        else:
            failed += 1
    if not ttw:
        return {"error": "no search won", "n": m}
    return {"p50": round(pct(ttw, 50) * 1e3, 3), "p99": round(pct(ttw, 99) * 1e3, 3),
            "mean": round(statistics.mean(ttw) * 1e3, 3), "n": len(ttw), "failed": failed,
            "rank_searches_cancelled": cancelled,
            "shared_cancel": words.path is not None,
            "nonces_per_search": round(nonces / m),
            "node_gnps": round(nonces / busy / 1e9, 4) if busy > 0 else None,
            "node_gnps_note": "nonces hashed by all ranks / sum over roots of the time until the root's last rank "
                              "returned (per-root barriers excluded): the node's rate on one root at a time",
            "note": f"one root at a time searched by all {world} ranks on disjoint strides (rank r from "
                    "start + r*2^64/N), the first win cancelling the others through a shared-memory word; "
                    "winner's search time at the C ABI; after the timed region, not part of value"}


def run_timed(search, stats, reset_stats, steps: int, warmup: int, rank: int, world: int, dist=None):
    """Warm up, then time exactly `steps` searches per rank bracketed by barriers; reduce over ranks.

    With several ranks on one node the world * steps timed searches come from one NodeQueue (search
    i of the job is root R_{1,000,000 + i} whichever rank draws it); a rank alone searches R_{1,000,000
    + s}, s < steps.  search(i) -> (seconds, nonces_hashed); stats() -> (kernel_ms, kernel_nonces,
    launches).  Returns the rank-0 view: (total_nonces, max_wall_s, all_ttw_s, kernel_ms,
    kernel_nonces, launches) with kernel_* summed over ranks."""
    base_idx = 1_000_000 * (rank + 1)
    for w in range(warmup):
        search(base_idx + 900_000 + w)
    reset_stats()
    one_node = int(os.environ.get("LOCAL_WORLD_SIZE", str(world))) == world
    queue = NodeQueue.create(dist, rank, world * steps) if (dist is not None and world > 1 and one_node) else None
    if dist is not None:
        dist.barrier()
    # npow_search returns only after its streams drained, so the GPU is idle at both barriers
    t0 = time.perf_counter()
    ttw, nonces = [], 0
    if queue is None:
        for s in range(steps):
            dt, n = search(base_idx + s)
            ttw.append(dt)
            nonces += n
    else:
        while (i := queue.draw()) is not None:
            dt, n = search(1_000_000 + i)
            ttw.append(dt)
            nonces += n
    if dist is not None:
        dist.barrier()
    wall = time.perf_counter() - t0
    if queue is not None:
        queue.close()
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


class SclkSampler:
    """Samples the shader clock of HIP device `dev` while the timed searches run (SURVEY.md §8(d):
    report the roofline against the clock measured during the run, too).  The current DPM level
    (the '*' line of the GPU's sysfs pp_dpm_sclk) is read every `period` seconds by a host thread;
    the card is found by the PCI bus id the HIP runtime reports.  Reading sysfs touches no GPU
    queue.  summary() is None when the file is unavailable."""

    def __init__(self, dev: int, period: float = 0.05, span: str = "over the warmup and timed searches"):
        self.samples, self.bus, self.path, self.span = [], None, None, span
        # the same card's hwmon power reading (microwatts) and its power cap, when readable: whether a
        # run sits at the power limit that lowers its clock ("Priority runs")
        self.power, self.pw_path, self.cap_w = [], None, None
        self.period, self._stop = period, threading.Event()
        try:
            hip = ctypes.CDLL("libamdhip64.so.7")
            buf = ctypes.create_string_buffer(64)
            if hip.hipDeviceGetPCIBusId(buf, ctypes.c_int(64), ctypes.c_int(dev)) == 0:
                self.bus = buf.value.decode().lower()
                for d in glob.glob("/sys/class/drm/card*/device"):
                    if os.path.basename(os.path.realpath(d)).lower() == self.bus and \
                            os.path.exists(os.path.join(d, "pp_dpm_sclk")):
                        self.path = os.path.join(d, "pp_dpm_sclk")
                        for h in sorted(glob.glob(os.path.join(d, "hwmon", "hwmon*"))):
                            for name in ("power1_average", "power1_input"):
                                if os.path.exists(os.path.join(h, name)):
                                    self.pw_path = os.path.join(h, name)
                                    break
                            try:
                                with open(os.path.join(h, "power1_cap")) as f:
                                    self.cap_w = int(f.read()) / 1e6
                            except (OSError, ValueError):
                                pass
                            if self.pw_path:
                                break
                        break
        except (OSError, AttributeError):
            self.path = None
        self._thread = threading.Thread(target=self._run, daemon=True)

    def _read(self):
        with open(self.path) as f:
            for ln in f:
                if ln.rstrip().endswith("*"):
                    return int(ln.split(":")[1].strip().split("M")[0])
        return None

    def _run(self):
        while not self._stop.is_set():
            try:
                v = self._read()
            except (OSError, ValueError, IndexError):
                return
            if v is not None:
                self.samples.append(v)
            if self.pw_path:
                try:
                    with open(self.pw_path) as f:
                        self.power.append(int(f.read()) / 1e6)
                except (OSError, ValueError):
                    self.pw_path = None
            self._stop.wait(self.period)

    def __enter__(self):
        if self.path:
            self._thread.start()
        return self

    def __exit__(self, *exc):
        self._stop.set()
        if self._thread.is_alive():
            self._thread.join()

    def summary(self):
        if not self.samples:
            return None
        return {"mean": round(statistics.mean(self.samples), 1), "min": min(self.samples),
                "max": max(self.samples), "samples": len(self.samples),
                "source": f"current level of pp_dpm_sclk of rank 0's GPU ({self.bus}), every "
                          f"{int(self.period * 1e3)} ms {self.span}"}

    def power_summary(self):
        if not self.power:
            return None
        return {"mean": round(statistics.mean(self.power), 1), "max": round(max(self.power), 1),
                "cap": self.cap_w, "samples": len(self.power),
                "source": f"hwmon {os.path.basename(self.pw_path or '')} of rank 0's GPU ({self.bus}) in W, with its "
                          "power1_cap, sampled with the clock (the sensor updates more slowly than the samples)"}


def _pmc(names=PMC_POOL):
    """(file name, contents) of the newest committed rocprofv3 PMC summary of the workload's dominant
    kernel (tools/pmc_bench.sh on that workload; FETCH_SIZE doubled per the gfx950 correction).  PMC
    needs the profiler around the process, so the bench reports the committed measurement; (None,
    None) if absent."""
    for name in names:
        try:
            with open(os.path.join(HERE, "profiles", name)) as f:
                return name, json.load(f)
        except (OSError, ValueError):
            continue
    return None, None


def _pmc_traffic(names=PMC_POOL):
    return (_pmc(names)[1] or {}).get("hbm_bytes_per_launch")


def pmc_nonces_per_dispatch(pmc, valu_per_iteration):
    """Nonces per dispatch implied by the PMC instruction count: SQ_INSTS_VALU per dispatch / the VALU
    instructions of one wave iteration (the stream + the loop's own) x 64 lanes."""
    if not pmc:
        return None
    c = pmc.get("counters_mean", {})
    if "SQ_INSTS_VALU" not in c:
        return None
    return c["SQ_INSTS_VALU"] / valu_per_iteration * 64


LOOP_VALU = 5.5  # the search loop's VALU per iteration besides the stream: 5, and 2 v_readlane at every 4th


def result_line(world, steps, warmup, tot_nonces, max_wall, all_ttw, kern_ms, kern_nonces, launches, parallelism=None):
    gnps = tot_nonces / max_wall / 1e9
    per_rank_kernel_s = kern_ms * 1e-3 / world
    mix = stream_mix()
    ex = mix["executed_int32_ops"]
    # achieved / frac: the int32 ops the shipped stream executes per nonce (its header's mix); the
    # algorithmic 2,232 of SURVEY.md §8(d) in achieved_algorithmic / frac_algorithmic -- the stream does
    # less than that (host precompute, round 12's dead half), so only the executed count bounds frac by 1
    achieved_alg = (kern_nonces / world) * OPS_PER_NONCE / per_rank_kernel_s / 1e12 if kern_ms > 0 else 0.0
    achieved = achieved_alg * ex / OPS_PER_NONCE
    build = build_sha16()
    prof = timed_region_profile(build)
    pmc_name, pmc = _pmc(PMC_POOL)
    pmc_npd = pmc_nonces_per_dispatch(pmc, mix["valu"] + LOOP_VALU)
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
            "searches_total": len(all_ttw),
            "parallelism": parallelism or (
                f"dp{world} (disjoint roots per GPU, no collective)" if world == 1 else
                f"dp{world} ({len(all_ttw)} searches drawn from one node-wide queue by {world} "
                "one-GPU ranks; disjoint roots, no collective)"),
        },
        "p50_ttw_ms": round(pct(all_ttw, 50) * 1e3, 3),
        # a p99 needs ~100 samples: fewer (the driver's 20 timed steps) report the maximum as such
        **({"p99_ttw_ms": round(pct(all_ttw, 99) * 1e3, 3)} if len(all_ttw) >= 100 else
           {"max_ttw_ms": round(max(all_ttw) * 1e3, 3)}),
        "mean_ttw_ms": round(statistics.mean(all_ttw) * 1e3, 3),
        "n_ttw": len(all_ttw),
        "gnps_per_gpu": round(gnps / world, 4),
        "build_sha16": build,
        "roofline": {
            "bound": "valu",
            "kernel": STREAM["kernel"],
            "achieved": round(achieved, 3),
            "peak": round(PEAK_TOPS, 3),
            "unit": "Tops/s (int32 VALU)",
            "frac": round(achieved / PEAK_TOPS, 4),
            "achieved_what": f"kernel-hashed nonces x {ex} int32 ops the shipped stream executes per nonce "
                             f"(executed_mix) / HIP-event-timed kernel time",
            "achieved_algorithmic": round(achieved_alg, 3),
            "frac_algorithmic": round(achieved_alg / PEAK_TOPS, 4),
            "algorithmic_note": f"the same nonces x {OPS_PER_NONCE} algorithmic ops per nonce (SURVEY.md §8d): the "
                                "stream executes fewer (round 1's three nonce-independent column steps on the host, "
                                "round 12's dead half removed), so this fraction can pass 1",
            "peak_note": "peak = 256 CUs x 4 SIMDs x 32 lanes x 2.4 GHz, one wave64 VALU instruction per 2 cycles "
                         "per SIMD (MI355X_MICROARCH.md).  gfx950 also issues a full-rate instruction of one wave "
                         "in the shadow of another wave's v_alignbit_b32 (tools/experiments/dual_issue.py; PMC "
                         "SQ_ACTIVE_INST_VALU2), which the stream's priority runs exploit; the GPU's power cap "
                         "holds its clock below 2.4 GHz meanwhile (sclk_mhz): issue_model holds the bound that "
                         "applies to this instruction mix",
            "profile": (dict(prof, recompute=f"frac = nonces_per_launch x {ex} / avg_dispatch_ms / {PEAK_TOPS:.3f} Tops/s; "
                                             "the fraction follows the box's power-limited clock, so compare "
                                             "cycles_per_hash_from_profile with issue_model.kernel_cycles_per_hash")
                        if prof else None),
            "traffic": (pmc or {}).get("hbm_bytes_per_launch"),
            "traffic_unit": "HBM bytes per launch, rocprofv3 FETCH_SIZE/WRITE_SIZE passes "
                            f"(profiles/{pmc_name}, tools/pmc_bench.sh); algorithmic bytes: 0",
            "ops_per_nonce": OPS_PER_NONCE,
            "ops_note": "algorithmic int32 ops of one 12-round compression (SURVEY.md §8d); the stream executes "
                        "fewer: host precompute of nonce-independent steps and round 12's dead half removed",
            "executed_ops_per_nonce": ex,
            "executed_mix": mix["mix"],
            "kernel_gnps": round(kern_nonces / (kern_ms * 1e-3) / 1e9, 4) if kern_ms > 0 else None,
            "avg_launch_ms": round(kern_ms / launches, 4) if launches else None,
            "nonces_per_launch": round(kern_nonces / launches) if launches else None,
            "pmc_nonces_per_dispatch": round(pmc_npd) if pmc_npd else None,
            "pmc_note": (f"profiles/{pmc_name}: SQ_INSTS_VALU per dispatch / ({mix['valu']} stream + {LOOP_VALU} "
                         "loop VALU per wave iteration) x 64 lanes; that run's own launches (its avg_launch_ms "
                         "and clock), to compare with nonces_per_launch") if pmc_npd else None,
            "launches": launches,
            "issue_model": {
                "kernel_cycles_per_hash": None,  # filled in once the in-kernel clock is known (add_clock)
                "bound_cycles_per_hash": round(issue_bound_cycles(mix) + 4 * LOOP_VALU / 2),
                "what": "SIMD cycles per 64-nonce wave-hash: the kernel's own (1,024 SIMDs x 64 x in-kernel clock / "
                        "kernel rate) against the issue bound of its instruction mix (one half-rate instruction "
                        "per quad-cycle; full-rate ones in pairs or in an alignbit's shadow; "
                        "tools/experiments/dual_issue.py).  Co-issue lets the kernel exceed one int32 op per lane "
                        "per cycle, so frac_at_measured_sclk can pass 1; the GPU is then power-bound and lowers "
                        "its clock (sclk_mhz)",
            },
        },
        "cpu_baseline": None,
    }


def _reduce(dist, nonces, wall, ttw, extra_sum=()):
    """Sum nonces (and extra_sum values) over ranks, max wall, gather ttw."""
    if dist is None:
        return nonces, wall, ttw, list(extra_sum)
    import torch
    v = torch.tensor([float(nonces)] + [float(x) for x in extra_sum], dtype=torch.float64)
    dist.all_reduce(v, op=dist.ReduceOp.SUM)
    w_t = torch.tensor([wall], dtype=torch.float64)
    dist.all_reduce(w_t, op=dist.ReduceOp.MAX)
    gathered = [None] * dist.get_world_size()
    dist.all_gather_object(gathered, ttw)
    return int(v[0]), float(w_t[0]), [x for g in gathered for x in g], [float(x) for x in v[1:]]


def workload_allgpus(eng, args, rank, world, dist):
    """One process, --gpus GPUs (default every visible one) on one root at a time: config 2 at N GPUs."""
    if world > 1:
        raise SystemExit("--workload allgpus runs in ONE process (it drives every GPU itself)")
    n_dev = args.gpus if args.gpus > 1 else eng.n_devices
    for d in range(n_dev):
        eng.reset_stats(d)
    node = inprocess_node_ttw(eng, n_dev, args.steps)
    ks = [eng.stats(d) for d in range(n_dev)]
    kern_ms, kern_nonces, launches = sum(k.kernel_ms for k in ks), sum(k.nonces for k in ks), sum(k.launches for k in ks)
    wall = node["nonces_per_search"] * node["n"] / (node["node_gnps"] * 1e9)
    line = result_line(n_dev, args.steps, 0, node["nonces_per_search"] * node["n"], wall,
                       [node["p50"] / 1e3] * 1, kern_ms, kern_nonces, launches,
                       parallelism=f"in-process x{n_dev} (first-win flag only, no collective)")
    line["node_ttw_ms"] = node
    line.pop("max_ttw_ms", None)
    line["p50_ttw_ms"], line["p99_ttw_ms"], line["mean_ttw_ms"], line["n_ttw"] = node["p50"], node["p99"], node["mean"], node["n"]
    line["scaling"] = "strong"
    line["config"]["workload"] = (f"BASELINE configs[1] at N={n_dev}: one root at a time searched by every GPU "
                                  "of the process on disjoint strides, first win across GPUs")
    return line


def workload_sweep(eng, args, rank, world, dist):
    """BASELINE config 3: every valid nonce of [0, 2^bits) for the fixture root, exact."""
    import json as _json
    with open(os.path.join(HERE, "tests", "golden", "sweep_2p36.json")) as f:
        fx = _json.load(f)
    root, thr = bytes.fromhex(fx["root"]), int(fx["threshold"], 16)
    count = 1 << args.sweep_bits
    per = count // world
    lo = rank * per
    n_here = per if rank < world - 1 else count - lo
    devs = range(1) if world > 1 else range(args.gpus)  # in one process: the range split over --gpus devices
    for d in devs:
        eng.reset_stats(d)
    if dist is not None:
        dist.barrier()
    t0 = time.perf_counter()
    hits = eng.sweep(root, thr, lo, n_here, device_mask=(1 << len(devs)) - 1, cap=1 << 16)
    wall = time.perf_counter() - t0
    ks = [eng.stats(d) for d in devs]
    nonces, wall, _, (kms, kn, nl) = _reduce(dist, n_here, wall, [], (sum(k.kernel_ms for k in ks),
                                                                     sum(k.nonces for k in ks),
                                                                     sum(k.launches for k in ks)))
    if dist is not None:
        gathered = [None] * world
        dist.all_gather_object(gathered, hits)
        hits = sorted(h for g in gathered for h in g)
    want = [int(h, 16) for h in fx["hits"] if int(h, 16) < count]
    line = result_line(max(world, len(devs)), 1, 0, nonces, wall, [wall], kms, kn, nl)
    pmc_name, pmc = _pmc(PMC_SWEEP)
    line["roofline"]["kernel"] = STREAM["sweep_kernel"]
    line["roofline"]["traffic"] = (pmc or {}).get("hbm_bytes_per_launch")
    line["roofline"]["traffic_unit"] = ("HBM bytes per launch, rocprofv3 FETCH_SIZE/WRITE_SIZE passes "
                                        f"(profiles/{pmc_name}, tools/pmc_bench.sh); algorithmic bytes: "
                                        "8 per hit")
    for k in ("pmc_nonces_per_dispatch", "pmc_note"):
        line["roofline"].pop(k, None)
    line["config"] = {"workload": f"BASELINE configs[2]: exhaustive sweep of [0, 2^{args.sweep_bits}) for the "
                                  "fixture root at fffffff800000000, ranks split the range",
                      "threshold": fx["threshold"], "count": count,
                      "parallelism": f"dp{world} (contiguous sub-ranges, no collective on the data path)"}
    line["hits"] = len(hits)
    line["hits_exact_vs_fixture"] = hits == want
    if hits != want:
        raise RuntimeError(f"sweep hit set differs from the fixture ({len(hits)} vs {len(want)})")
    return line


def _burst_http(eng, args, rank, world, dist):
    """BASELINE config 4 at the JSON boundary: --roots concurrent work_generate POSTs to the HTTP
    work server (one connection each), 25 % answered by a work_cancel POST at a uniform time in
    [0, 0.5 x the expected burst time); every work reply re-validated (npow_work_value), every
    cancelled request must answer {"error": "Cancelled"} unless its work was already found."""
    import random
    import threading
    import urllib.request
    from nanopow.server import HttpWorkServer, WorkServer
    n = args.roots
    rng = random.Random(4343 + rank)
    idx = [9_000_000 + rank * 1_000_000 + i for i in range(n)]
    roots = [bench_root(i) for i in idx]
    cancel_set = set(rng.sample(range(n), n // 4))
    est = n * float(1 << 29) / (25e9 * max(1, eng.n_devices if world == 1 else 1))
    cancel_at = sorted((rng.uniform(0.0, 0.5 * est), i) for i in cancel_set)
    srv = HttpWorkServer(WorkServer(eng, max_active=64, device_mask=(1 << args.gpus) - 1 if world == 1 else 1), "127.0.0.1", 0).start()

    def post(obj, timeout=600):
        req = urllib.request.Request(f"http://{srv.address}", data=json.dumps(obj).encode(), method="POST",
                                     headers={"Content-Type": "application/json"})
        with urllib.request.urlopen(req, timeout=timeout) as r:
            return json.loads(r.read())
    replies, done_at = [None] * n, [0.0] * n
    eng.reset_stats(0)
    if dist is not None:
        dist.barrier()
    t0 = time.perf_counter()

    def client(i):
        replies[i] = post({"action": "work_generate", "hash": roots[i].hex().upper(), "difficulty": f"{SEND:016x}"})
        done_at[i] = time.perf_counter() - t0

    finished = threading.Event()

    def canceller():
        for t_c, i in cancel_at:
            if finished.wait(max(0.0, t0 + t_c - time.perf_counter())):
                return  # every request has been answered
            post({"action": "work_cancel", "hash": roots[i].hex().upper()})
    try:
        ths = [threading.Thread(target=client, args=(i,)) for i in range(n)]
        for t in ths:
            t.start()
        th_c = threading.Thread(target=canceller, daemon=True)
        th_c.start()
        for t in ths:
            t.join()
        wall = time.perf_counter() - t0
        finished.set()
        th_c.join(60)
    finally:
        srv.stop()
    ok = [i for i in range(n) if "work" in replies[i]]
    bad = [i for i in ok if eng.work_value(roots[i], int(replies[i]["work"], 16)) < SEND]
    wrong_err = [i for i in range(n) if "work" not in replies[i]
                 and (i not in cancel_set or replies[i].get("error") != "Cancelled")]
    st = eng.stats(0)
    ttw = [done_at[i] for i in ok]
    nonces, wall, ttw, (kms, kn, nl, n_bad, n_we) = _reduce(dist, st.nonces, wall, ttw,
                                                            (st.kernel_ms, st.nonces, st.launches, len(bad),
                                                             len(wrong_err)))
    line = result_line(world, n, 0, nonces, wall, ttw or [0.0], kms, kn, nl)
    line["config"] = {"workload": f"BASELINE configs[3]: burst of {n} concurrent work_generate requests per GPU "
                                  "at fffffff800000000 POSTed to the HTTP work server, 25 % answered by work_cancel",
                      "threshold": "fffffff800000000", "roots_per_gpu": n, "boundary": "JSON over HTTP (127.0.0.1)",
                      "parallelism": f"dp{world} (disjoint roots per GPU)" if world > 1 else
                                     f"work pool over {eng.n_devices} GPU(s)"}
    line["burst"] = {"ok": len(ok), "cancelled_requested": len(cancel_set),
                     "cancel_lost_race": sum(1 for i in cancel_set if "work" in replies[i]),
                     "invalid_replies": int(n_bad), "unexpected_errors": int(n_we)}
    if n_bad or n_we:
        raise RuntimeError(f"burst/http: {int(n_bad)} invalid replies, {int(n_we)} unexpected errors")
    return line


def workload_burst(eng, args, rank, world, dist):
    """BASELINE config 4: a burst of --roots concurrent requests with 25 % mid-search cancels."""
    import queue
    import random
    import threading
    from nanopow import _lib
    if args.via == "http":
        return _burst_http(eng, args, rank, world, dist)
    n = args.roots
    rng = random.Random(4242 + rank)
    idx = [7_000_000 + rank * 1_000_000 + i for i in range(n)]
    roots = [bench_root(i) for i in idx]
    toks = [_lib.CancelToken() for _ in range(n)]
    cancel_set = set(rng.sample(range(n), n // 4))
    est = n * float(1 << 29) / (25e9 * max(1, eng.n_devices if world == 1 else 1))
    cancel_at = sorted((rng.uniform(0.0, 0.5 * est), i) for i in cancel_set)
    eng.reset_stats(0)
    if dist is not None:
        dist.barrier()
    t0 = time.perf_counter()
    tickets = [eng.submit(roots[i], SEND, start=bench_start(idx[i]), device_mask=(1 << args.gpus) - 1 if world == 1 else 1,
                          cancel=toks[i]) for i in range(n)]

    def canceller():
        for t_c, i in cancel_at:
            dt = t0 + t_c - time.perf_counter()
            if dt > 0:
                time.sleep(dt)
            toks[i].set()
    th_c = threading.Thread(target=canceller, daemon=True)
    th_c.start()
    q: "queue.Queue[int]" = queue.Queue()
    for i in range(n):
        q.put(i)
    done_at, results = [0.0] * n, [None] * n

    def waiter():
        while True:
            try:
                i = q.get_nowait()
            except queue.Empty:
                return
            results[i] = tickets[i].wait()
            done_at[i] = time.perf_counter() - t0
    ws = [threading.Thread(target=waiter) for _ in range(64)]
    for w in ws:
        w.start()
    for w in ws:
        w.join()
    wall = time.perf_counter() - t0
    th_c.join(0)
    ok = [i for i in range(n) if results[i].status == 0]
    bad = [i for i in ok if eng.work_value(roots[i], results[i].nonce) != results[i].value
           or results[i].value < SEND]
    unc_fail = [i for i in range(n) if i not in cancel_set and results[i].status != 0]
    canc_ok = sum(1 for i in cancel_set if results[i].status == 0)
    nonces = sum(r.nonces_done for r in results)
    ttw = [done_at[i] for i in ok]
    st = eng.stats(0)
    nonces, wall, ttw, (kms, kn, nl, n_bad, n_uf) = _reduce(dist, nonces, wall, ttw,
                                                            (st.kernel_ms, st.nonces, st.launches, len(bad),
                                                             len(unc_fail)))
    line = result_line(world, n, 0, nonces, wall, ttw or [0.0], kms, kn, nl)
    line["config"] = {"workload": f"BASELINE configs[3]: burst of {n} concurrent requests per GPU at "
                                  "fffffff800000000 through the work pool, 25 % cancelled mid-search",
                      "threshold": "fffffff800000000", "roots_per_gpu": n,
                      "parallelism": f"dp{world} (disjoint roots per GPU)" if world > 1 else
                                     f"work pool over {eng.n_devices} GPU(s)"}
    line["burst"] = {"ok": len(ok), "cancelled_requested": len(cancel_set),
                     "cancel_lost_race": canc_ok, "invalid_replies": int(n_bad),
                     "uncancelled_failures": int(n_uf)}
    if n_bad or n_uf:
        raise RuntimeError(f"burst: {int(n_bad)} invalid replies, {int(n_uf)} uncancelled failures")
    return line


def workload_sustained(eng, args, rank, world, dist):
    """BASELINE config 5: --duration seconds of fresh roots, --depth requests in flight per GPU."""
    eng.reset_stats(0)
    if dist is not None:
        dist.barrier()
    t0 = time.perf_counter()
    pending = []
    nxt, nonces, ttw = 0, 0, []
    base = 9_000_000 + rank * 10_000_000
    # every request is replaced as soon as it returns, whichever finishes first (polled every 0.2 ms:
    # a FIFO wait on the oldest would leave the others' slots empty and count their queueing as ttw)
    while True:
        now = time.perf_counter()
        while len(pending) < args.depth and now - t0 < args.duration:
            i = base + nxt
            nxt += 1
            pending.append((eng.submit(bench_root(i), SEND, start=bench_start(i), device_mask=1), now))
        if not pending:
            break
        still = []
        for t, ts in pending:
            r = t.wait(0)
            if r is None:
                still.append((t, ts))
                continue
            if r.status != 0:
                raise RuntimeError(f"sustained: status {r.status}")
            nonces += r.nonces_done
            ttw.append(time.perf_counter() - ts)
        if len(still) == len(pending):
            time.sleep(0.0002)
        pending = still
    wall = time.perf_counter() - t0
    st = eng.stats(0)
    nonces, wall, ttw, (kms, kn, nl) = _reduce(dist, nonces, wall, ttw, (st.kernel_ms, st.nonces, st.launches))
    line = result_line(world, len(ttw), 0, nonces, wall, ttw, kms, kn, nl)
    line["config"] = {"workload": f"BASELINE configs[4]: {args.duration:.0f} s of back-to-back fresh roots at "
                                  f"fffffff800000000, {args.depth} in flight per GPU",
                      "threshold": "fffffff800000000", "duration_s": args.duration, "depth": args.depth,
                      "parallelism": f"dp{world} (per-GPU roots and strides, no collective)"}
    return line


def workload_dpow(eng, args, rank, world, dist):
    """MQTT path: work/cancel messages -> WorkHandler-equivalent -> HTTP server -> results."""
    import asyncio
    import random
    from nanopow import dpow
    from nanopow.server import HttpWorkServer, WorkServer
    n = args.roots
    rng = random.Random(777 + rank)
    srv = HttpWorkServer(WorkServer(eng, max_active=max(1, args.concurrency), device_mask=(1 << args.gpus) - 1 if world == 1 else 1),
                         "127.0.0.1", 0).start()
    hashes = [bench_root(11_000_000 + rank * 1_000_000 + i).hex().upper() for i in range(n)]
    t, sched = 0.0, []
    for h in hashes:
        t += rng.expovariate(args.rate)
        sched.append((t, "work/ondemand", f"{h},fffffff800000000".encode()))
    cancelled = set(rng.sample(range(n), n // 4))
    for i in cancelled:
        sched.append((sched[i][0] + rng.uniform(0.0, 0.05), "cancel/ondemand", hashes[i].encode()))
    published = []

    async def main():
        probe = dpow.LatencyProbe()

        async def publish(topic, payload):
            published.append((topic, payload))
            probe.saw_result(topic, payload)
        h = dpow.DpowWorkHandler(dpow.HttpWorker(srv.address, timeout=120), publish, "nano_bench",
                                 concurrency=args.concurrency, rng=random.Random(rank))
        await h.start()
        wall = await dpow.replay(h, probe, sched, drain_timeout=300)
        await h.stop()
        return probe, wall
    eng.reset_stats(0)
    if dist is not None:
        dist.barrier()
    try:
        probe, wall = asyncio.run(main())
    finally:
        srv.stop()
    bad = 0
    for _, payload in published:
        bh, work, _ = payload.decode().split(",")
        if eng.work_value(bytes.fromhex(bh), int(work, 16)) < SEND:
            bad += 1
    lat = [probe.latency[h] for h in probe.latency]
    st = eng.stats(0) if world > 1 else None
    if world == 1:
        ks = [eng.stats(d) for d in range(eng.n_devices)]
        kms, kn, nl = sum(k.kernel_ms for k in ks), sum(k.nonces for k in ks), sum(k.launches for k in ks)
    else:
        kms, kn, nl = st.kernel_ms, st.nonces, st.launches
    nonces, wall, lat, (kms, kn, nl, n_bad) = _reduce(dist, kn, wall, lat, (kms, kn, nl, bad))
    line = result_line(world, len(lat), 0, nonces, wall, lat or [0.0], kms, kn, nl)
    line["config"] = {"workload": f"MQTT path end to end: {n} work messages per GPU at fffffff800000000, "
                                  f"Poisson arrivals at {args.rate}/s, 25 % cancelled, WorkHandler-equivalent "
                                  f"with {args.concurrency} loop(s) -> HTTP work server -> engine",
                      "threshold": "fffffff800000000", "rate_per_s": args.rate, "concurrency": args.concurrency,
                      "parallelism": f"dp{world}" if world > 1 else f"work pool over {eng.n_devices} GPU(s)"}
    line["dpow"] = {"results": len(published), "cancelled": len(cancelled), "invalid_results": int(n_bad)}
    line["value_note"] = "value = nonces hashed by the kernels / wall time of the whole message stream (idle included)"
    if n_bad:
        raise RuntimeError(f"dpow: {int(n_bad)} invalid results")
    return line


def _hashlib_search(root: bytes, thr: int, start: int, limit: int):
    """The reference's CPU path: hashlib.blake2b(digest_size=8) over consecutive nonces."""
    b2 = hashlib.blake2b
    n = start
    for k in range(limit):
        if int.from_bytes(b2(n.to_bytes(8, "little") + root, digest_size=8).digest(), "little") >= thr:
            return k + 1, n
        n = (n + 1) & ((1 << 64) - 1)
    return limit, None


class KeepAliveClient:
    """One persistent HTTP/1.1 connection to the work server, as the DPoW client's aiohttp session
    keeps one for its serial work_generate loop (client/work_handler.py:98-108).  A lean client: one
    send per request (TCP_NODELAY), the reply read by its Content-Length -- aiohttp parses with a C
    parser, while http.client's Python header parsing added ~0.3 ms per request on this container and
    stood in the measured HTTP hop (round 5, tools/experiments/http_hop.py)."""

    def __init__(self, address: str):
        import socket
        host, port = address.rsplit(":", 1)
        self.sock = socket.create_connection((host, int(port)), timeout=120)
        self.sock.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        self.buf = b""

    def post(self, obj):
        body = json.dumps(obj).encode()
        self.sock.sendall(b"POST / HTTP/1.1\r\nHost: localhost\r\nContent-Type: application/json\r\n"
                          b"Content-Length: %d\r\n\r\n" % len(body) + body)
        while b"\r\n\r\n" not in self.buf:
            self._recv()
        head, _, rest = self.buf.partition(b"\r\n\r\n")
        lines = head.split(b"\r\n")
        if not lines[0].startswith(b"HTTP/1.1 200"):
            raise RuntimeError(f"HTTP reply {lines[0]!r}")
        n = next(int(v) for k, _, v in (h.partition(b":") for h in lines[1:]) if k.strip().lower() == b"content-length")
        while len(rest) < n:
            self.buf = rest
            self._recv()
            rest = self.buf
        self.buf = rest[n:]
        return json.loads(rest[:n])

    def _recv(self):
        d = self.sock.recv(65536)
        if not d:
            raise RuntimeError("the work server closed the connection")
        self.buf += d

    def close(self):
        self.sock.close()


def _http_ttw(eng, n, thr=SEND, base=30_000_000, device_mask=1):
    """A config at the JSON boundary: n work_generate requests POSTed one at a time over one
    keep-alive connection to the HTTP work server on 127.0.0.1 (fresh roots); wall time per
    POST -> reply, each reply re-validated through npow_work_value."""
    from nanopow.server import HttpWorkServer, WorkServer
    srv = HttpWorkServer(WorkServer(eng, max_active=1, device_mask=device_mask), "127.0.0.1", 0).start()
    cli = KeepAliveClient(srv.address)
    out = []
    try:
        for i in range(n):
            root = bench_root(base + i)
            t = time.perf_counter()
            rep = cli.post({"action": "work_generate", "hash": root.hex().upper(), "difficulty": f"{thr:016x}"})
            out.append(time.perf_counter() - t)
            if eng.work_value(root, int(rep["work"], 16)) < thr:
                raise RuntimeError(f"HTTP reply {rep} does not validate")
    finally:
        cli.close()
        srv.stop()
    return out


def fixed_overhead(eng, mask: int, rate: float, n: int = 300):
    """The per-search cost that does not scale with nonces: n receive-difficulty searches (2^23 nonces
    expected, ~0.25 ms of hashing) through the C ABI, one at a time; per search, its wall time minus
    its nonces at the kernel rate -- submit, adopt, launch, the cold first hash, the win seen and
    re-validated, the launch drained, the reply.  (Threshold 0 is no measure of it: every wave of the
    first hash wins, and 8,192 win atomics on one word serialise for ~0.15 ms.)"""
    res, ts = [], []
    for i in range(n):
        dt, _t_all, info = search_to_result(eng, bench_root(40_000_000 + i), 0xfffffe0000000000, bench_start(i), mask)
        ts.append(dt)
        res.append(dt - info.nonces_done / rate)
    return {"p50": round(pct(res, 50) * 1e3, 4), "mean": round(statistics.mean(res) * 1e3, 4), "n": n,
            "receive_p50_ms": round(pct(ts, 50) * 1e3, 4),
            "how": "receive-difficulty searches (fffffe00...) one at a time: wall time - nonces_done / kernel rate"}


def latency_sample(eng, dev: int, n: int, rate_gnps=None, snap=None):
    """BASELINE config 2's time-to-work on a real sample: n first-win searches on R_0..R_{n-1} at
    fffffff8 through the C ABI, one at a time, after the timed region (not part of value), with the
    decomposition of its p50 / mean: the sample's own nonce counts against the exponential law's
    (E = 2^29, median ln2 * 2^29), the fixed per-search overhead, and the kernel rate.  snap (optional):
    called right after the n searches, before the overhead sample; its result is returned as out["_snap"]."""
    ttw, nn, coll = [], [], []
    t0 = time.perf_counter()
    for i in range(n):
        t_res, t_all, info = search_to_result(eng, bench_root(i), SEND, bench_start(i), 1 << dev)
        ttw.append(t_res)
        coll.append(t_all)
        nn.append(info.nonces_done)
    wall = time.perf_counter() - t0
    snapped = snap() if snap else None
    E = float(1 << 29)
    ln2 = 0.6931471805599453
    mean_n = statistics.mean(nn)
    se_n = statistics.stdev(nn) / n ** 0.5 if n > 1 else 0.0
    rate = (rate_gnps or sum(nn) / wall / 1e9) * 1e9  # nonces / s
    over = fixed_overhead(eng, 1 << dev, rate)
    oh = over["p50"] * 1e-3
    out = {"p50": round(pct(ttw, 50) * 1e3, 3), "p99": round(pct(ttw, 99) * 1e3, 3),
           "mean": round(statistics.mean(ttw) * 1e3, 3), "n": n, "gnps": round(sum(nn) / wall / 1e9, 4),
           "collected_p50": round(pct(coll, 50) * 1e3, 3),
           "what": "submit -> npow_wait_result (the winner accepted: what a client is answered with); "
                   "collected_p50: -> npow_wait_info (the device stopped, nonces_done complete)",
           "roots": f"R_0..R_{n - 1}",
           "nonces_per_search": {
               "mean_over_2p29": round(mean_n / E, 4), "se_over_2p29": round(se_n / E, 4),
               "median_over_ln2_2p29": round(pct(nn, 50) / (ln2 * E), 4),
               "note": "nonces_done of each search (the winner's launch drains one hash after the win: ~0.5 M "
                       "nonces, 0.1 % of 2^29); an exponential law has mean 2^29 and median ln2 * 2^29"},
           "fixed_overhead_ms": over,
           "model": {
               "rate_gnps": round(rate / 1e9, 4),
               "expected_p50_ms": round((ln2 * E / rate + oh) * 1e3, 3),
               "expected_mean_ms": round((E / rate + oh) * 1e3, 3),
               "p50_from_sample_nonces_ms": round((pct(nn, 50) / rate + oh) * 1e3, 3),
               "mean_from_sample_nonces_ms": round((mean_n / rate + oh) * 1e3, 3),
               "what": "time = fixed overhead + nonces / kernel rate: expected_* use the exponential law's "
                       "nonces, *_from_sample_nonces the sample's own; the gap between p50 and expected_p50 "
                       "that p50_from_sample_nonces closes is the sample's luck, the rest is per-search cost"},
           "note": "npow_search at fffffff800000000 through the C ABI, one at a time, after the timed region; "
                   "not part of value"}
    if snapped is not None:
        out["_snap"] = snapped
    return out


def steady_state(lat, leg, sampler, n):
    """the rate at the card's power-capped steady state, beside the headline.  The driver's timed
    region is ~0.2 s (20 searches) -- the card has not reached its power cap yet -- while the time-to-work leg runs
    ~11 s of the same searches: value_steady = its nonces / its wall time (value's definition), with the kernel-counted
    rate, the in-kernel clock of the same launches, the card's power, and the roofline fraction at 2.4 GHz and at
    that clock (executed int32 ops, as roofline.frac)."""
    ex = stream_mix()["executed_int32_ops"]
    kg = leg.nonces / (leg.kernel_ms * 1e-3) / 1e9 if leg.kernel_ms > 0 else None
    mhz = leg.clock_mhz or None
    achieved = kg * ex / 1e3 if kg else None  # Tops/s
    pw = sampler.power_summary()
    return {"value": lat["gnps"], "unit": "Gnonce/s",
            "kernel_gnps": round(kg, 4) if kg else None,
            "in_kernel_mhz": round(mhz, 1) if mhz else None,
            "frac": round(achieved / PEAK_TOPS, 4) if achieved else None,
            "frac_at_measured_sclk": round(achieved / (256 * 128 * mhz * 1e6 / 1e12), 4) if achieved and mhz else None,
            "power_w": pw,
            "cycles_per_hash": round(1024 * 64 * mhz * 1e6 / (kg * 1e9), 1) if kg and mhz else None,
            "joules_per_gnonce": round(pw["mean"] / lat["gnps"], 2) if pw and lat.get("gnps") else None,
            "what": f"the {n} time-to-work searches at fffffff8 after the timed region (ttw_c_abi_ms; ~11 s, the card "
                    "at its power-capped steady state): value = their nonces / their wall time (the headline's "
                    "definition), kernel_gnps = the kernels' count / their HIP-event time, frac = kernel rate x "
                    f"{ex} executed int32 ops / 78.64 Tops/s (2.4 GHz) and at the in-kernel clock of those launches"}


def run_timed_inprocess(eng, n_dev: int, steps: int, warmup: int, thr: int = SEND):
    """The product's own multi-GPU path in one process: the work pool over device_mask = the first
    n_dev devices, n_dev searches in flight (one per client thread, each blocked in npow_wait_info
    with the GIL released), every search split into n_dev disjoint strides with first-found
    cancellation across the GPUs.  n_dev * steps timed searches on R_{1,000,000 + i}.  Returns
    (nonces, wall_s, ttw_s list, infos, kernel_ms summed over devices, kernel nonces, launches)."""
    mask = (1 << n_dev) - 1
    for w in range(warmup):
        eng.submit(bench_root(1_900_000 + w), thr, start=bench_start(1_900_000 + w), device_mask=mask).wait()
    for d in range(n_dev):
        eng.reset_stats(d)
    total = n_dev * steps
    lock = threading.Lock()
    nxt = [0]
    recs = []
    errors = []

    def client():
        while True:
            with lock:
                i = nxt[0]
                if i >= total:
                    return
                nxt[0] += 1
            idx = 1_000_000 + i
            try:
                t = time.perf_counter()
                info = eng.submit(bench_root(idx), thr, start=bench_start(idx), device_mask=mask).wait_info()
                dt = time.perf_counter() - t
            except Exception as e:  # reported after the join
                errors.append(repr(e))
                return
            if info.status != 0:
                errors.append(f"search {idx} returned status {info.status}")
                return
            with lock:
                recs.append((dt, info.nonces_done, info.stop_after_decide_us, info.overshoot_nonces,
                             info.late_nonces_losers))
    t0 = time.perf_counter()
    ths = [threading.Thread(target=client) for _ in range(n_dev)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    wall = time.perf_counter() - t0
    if errors:
        raise RuntimeError("; ".join(errors[:4]))
    ks = [eng.stats(d) for d in range(n_dev)]
    return (sum(r[1] for r in recs), wall, [r[0] for r in recs], recs, sum(k.kernel_ms for k in ks),
            sum(k.nonces for k in ks), sum(k.launches for k in ks), ks)


def busy_ms(k) -> float:
    """A device's HIP-event kernel time less what its lingering launches spent waiting with nothing to hash
    (npow_device_stats.linger_ms, ABI 6; 0 from older libraries): the time it hashed."""
    return max(0.0, k.kernel_ms - getattr(k, "linger_ms", 0.0))


def hash_rate(k) -> float:
    """Nonces per second over the time the device hashed (busy_ms); 0 before its first launch."""
    b = busy_ms(k)
    return k.nonces / (b * 1e-3) if b > 0 else 0.0


def device_check(rates, kernel_nonces, search_nonces, clocks=None):
    """a multi-GPU run fails loudly rather than reporting a node rate with a slow or miscounting
    device in it -- every device's kernel rate within 0.9x of the median, and the devices' nonce counters
    (npow_device_stats) summing exactly to the nonces the searches report (nonces_done).  With each device's
    in-kernel clock known, the rate is compared per MHz: every GPU's own power cap sets its clock (2,170-2,340
    MHz across this pool's boxes, 0.93x), which is no fault, while a device hashing slowly at its clock is."""
    per = ([r / c for r, c in zip(rates, clocks)] if clocks and len(clocks) == len(rates) and all(c > 0 for c in clocks)
           else None)
    basis = per if per is not None else rates
    med = statistics.median(basis) if basis else 0.0
    slow = [i for i, r in enumerate(basis) if r < 0.9 * med]
    out = {"ok": not slow and kernel_nonces == search_nonces,
           "kernel_gnps": [round(r, 4) for r in rates], "median_gnps": round(statistics.median(rates), 4) if rates else 0.0,
           "slow_devices": slow, "kernel_nonces": int(kernel_nonces), "search_nonces": int(search_nonces),
           "what": "each device's kernel rate (per MHz of its in-kernel clock when known) >= 0.9 x the median, and "
                   "the device counters' nonces == the searches' nonces_done; bench.py exits non-zero otherwise"}
    if per is not None:
        out["in_kernel_mhz"] = [round(c, 1) for c in clocks]
        out["mnonce_per_s_per_mhz"] = [round(x * 1e3, 3) for x in per]
    return out


def overshoot_summary(spans_us, over_nonces, done, late=None):
    out = {"stop_after_decide_us": {"p50": round(pct(spans_us, 50), 1), "p99": round(pct(spans_us, 99), 1)},
           "overshoot_nonces": {"p50": int(pct(over_nonces, 50)), "p99": int(pct(over_nonces, 99)),
                                "share_of_nonces": round(sum(over_nonces) / max(1, sum(done)), 5)},
           "what": "per search, how long the other GPUs kept hashing after the host accepted the winner "
                   "(host-observed: their final count or launch end seen by their worker -- an upper bound) "
                   "and the nonces that span is worth at each GPU's kernel rate (npow_wait_info)"}
    if late is not None:
        # counted in the kernels: the losers' hashes for the job after one of their waves knew it was over.  With
        # several jobs in a launch the workgroups that leave a dead entry go on hashing the others, so the
        # host-observed span above is mostly useful work; this is the waste
        out["late_nonces_losers"] = {"p50": int(pct(late, 50)), "p99": int(pct(late, 99)),
                                     "share_of_nonces": round(sum(late) / max(1, sum(done)), 6)}
    return out


def inprocess_node_ttw(eng, n_dev: int, m: int, thr: int = SEND):
    """One root at a time over all n_dev devices of the process (north_star: the nonce space split
    into disjoint per-GPU strides, first found cancels the others): p50/p99 time-to-work at N GPUs
    and each search's overshoot (npow_wait_info)."""
    mask = (1 << n_dev) - 1
    ttw, spans, over, done, decide, fin, late = [], [], [], [], [], [], []
    t0 = time.perf_counter()
    for i in range(m):
        idx = 3_000_000 + i
        t_res, t_all, info = search_to_result(eng, bench_root(idx), thr, bench_start(idx), mask)
        ttw.append(t_res)
        fin.append(t_all)
        spans.append(info.stop_after_decide_us)
        over.append(info.overshoot_nonces)
        done.append(info.nonces_done)
        decide.append(info.decide_us)
        late.append(info.late_nonces_losers)
    wall = time.perf_counter() - t0
    return {"p50": round(pct(ttw, 50) * 1e3, 3), "p99": round(pct(ttw, 99) * 1e3, 3),
            "mean": round(statistics.mean(ttw) * 1e3, 3), "n": m, "node_gnps": round(sum(done) / wall / 1e9, 4),
            "decide_p50_ms": round(pct(decide, 50) / 1e3, 3),
            "collected_p50_ms": round(pct(fin, 50) * 1e3, 3),
            "late_nonces_losers_p50": int(pct(late, 50)),
            "nonces_per_search": round(statistics.mean(done)),
            **overshoot_summary(spans, over, done),
            "note": f"one root at a time searched by all {n_dev} GPUs of the process on disjoint strides "
                    "(npow_submit over device_mask), first win cancelling the others; after the timed region, "
                    "not part of value"}


REGIME = 0xffffffc000000000  # 2^-26 per nonce: fffffff8's 2^29 nonces split over 8 GPUs, on one GPU's rate


def _mean_p(xs):
    xs = [x for x in xs if x is not None]
    if not xs:
        return None
    return {"mean": round(statistics.mean(xs), 1), "p50": round(pct(xs, 50), 1), "p99": round(pct(xs, 99), 1)}


def node_regime(eng, n_dev: int, m: int, thr: int = REGIME, http_m: int = 0):
    """the 8-GPU time regime on the devices of this process.  One root at a time over all n_dev
    devices (disjoint strides, first win cancels the others), as the DPoW client's serial loop sends them
    (client/work_handler.py:98-125): the next root is submitted as soon as the previous result is in (npow_wait_result,
    what a client is answered with), and a reaper thread collects each ticket behind it (npow_wait_info: nonces and
    timeline), as the JSON server does.  At ffffffc0 a search expects 2^26 nonces: ~1.9 ms on one MI355X, the time
    scale of fffffff8 (2^29) on 8 GPUs -- so per-search fixed costs weigh what they would there.

    Reports the C-ABI time-to-work against ln2 * 2^26 / the node's kernel rate, the node's rate against its kernel
    rate, and the per-search fixed cost decomposed: the GPU idle between searches (HIP events), the host timeline of
    each search (adopt, launch issue on the first / last device, the winner's record read, the decision, the result
    in the client), the client's turnaround to the next submit, the losers' stop; optionally http_m requests over
    one keep-alive connection (the HTTP hop)."""
    import queue
    mask = (1 << n_dev) - 1
    # The devices' full rate, for reference (round 5): one search that cannot end (threshold 2^64 - 1) over every
    # device, cancelled after 0.4 s -- nonces / wall.  With lingering launches (a launch waits in the GPU for the next
    # search) the kernels' event time includes the waits between searches, so the kernel rate below is no longer
    # the rate the devices hash at; this is.
    t_ref = time.perf_counter()
    tk_ref = eng.submit(bench_root(6_950_000), (1 << 64) - 1, start=0, device_mask=mask)
    time.sleep(0.4)
    tk_ref.cancel()
    ref_info = tk_ref.wait_info()
    ref_rate = ref_info.nonces_done / (time.perf_counter() - t_ref)
    for w in range(5):
        search_to_result(eng, bench_root(6_900_000 + w), thr, bench_start(w), mask)
    for d in range(n_dev):
        eng.reset_stats(d)
    q: "queue.Queue" = queue.Queue()
    infos, errors = [], []

    def reaper():
        while True:
            item = q.get()
            if item is None:
                return
            try:
                infos.append(item.wait_info())
            except Exception as e:  # reported below
                errors.append(repr(e))
    th = threading.Thread(target=reaper, daemon=True)
    th.start()
    res, turn = [], []
    t0 = time.perf_counter()
    t_prev = None
    for i in range(m):
        idx = 6_000_000 + i
        root = bench_root(idx)
        t = time.perf_counter()
        if t_prev is not None:
            turn.append((t - t_prev) * 1e6)  # the client's turnaround: result in hand -> the next submit
        tk = eng.submit(root, thr, start=bench_start(idx), device_mask=mask)
        r = tk.wait_result()
        t_prev = time.perf_counter()
        if r is None or r.status != 0 or eng.work_value(root, r.nonce) != r.value or r.value < thr:
            raise RuntimeError(f"regime search {idx}: bad result {r}")
        res.append(t_prev - t)
        q.put(tk)
    q.put(None)
    th.join()
    wall = time.perf_counter() - t0
    if errors:
        raise RuntimeError("; ".join(errors[:4]))
    ks = [eng.stats(d) for d in range(n_dev)]
    done = [x.nonces_done for x in infos]
    kern_rate = sum(hash_rate(k) for k in ks)  # node: devices side by side (lingering waits left out: busy_ms)
    node_gnps = sum(done) / wall / 1e9
    ln2 = 0.6931471805599453
    E = float(1 << 64) / float((1 << 64) - thr)
    per_search_us = wall / m * 1e6
    hashing_us = statistics.mean(done) / kern_rate * 1e6
    idle = [k.idle_ms * 1e3 / k.idle_gaps for k in ks if k.idle_gaps]
    line = {
        "threshold": f"{thr:016x}", "devices": n_dev, "searches": m,
        "c_abi_ttw_ms": {"p50": round(pct(res, 50) * 1e3, 4), "p99": round(pct(res, 99) * 1e3, 4),
                         "mean": round(statistics.mean(res) * 1e3, 4)},
        "kernel_gnps": round(kern_rate / 1e9, 4),
        "node_gnps": round(node_gnps, 4),
        "node_over_kernel": round(node_gnps * 1e9 / kern_rate, 4),
        "reference_gnps": round(ref_rate / 1e9, 4),
        "node_over_reference": round(node_gnps * 1e9 / ref_rate, 4),
        "p50_minus_expected_at_reference_ms": round(pct(res, 50) * 1e3 - ln2 * E / ref_rate * 1e3, 4),
        "reference_what": "every device on one search that cannot end, cancelled after 0.4 s: its nonces / wall -- "
                          "the devices' full rate; with lingering launches the kernel rate above (HIP events) "
                          "includes the launches' waits for the next search",
        "expected_p50_ms": round(ln2 * E / kern_rate * 1e3, 4),
        "expected_mean_ms": round(E / kern_rate * 1e3, 4),
        "p50_minus_expected_ms": round(pct(res, 50) * 1e3 - ln2 * E / kern_rate * 1e3, 4),
        "nonces_per_search_over_E": round(statistics.mean(done) / E, 4),
        "fixed_cost_at_reference_us": round(per_search_us - statistics.mean(done) / ref_rate * 1e6, 1),
        "fixed_cost_us": {
            "per_search_wall_us": round(per_search_us, 1),
            "hashing_at_kernel_rate_us": round(hashing_us, 1),
            "fixed_us": round(per_search_us - hashing_us, 1),
            "what": "wall time per search minus its nonces at the node's kernel rate: what the parts below make up"},
        "decomposition_us": {
            "gpu_idle_between_launches": {
                "mean_per_gap": round(statistics.mean(idle), 1) if idle else None,
                "per_device": [round(x, 1) for x in idle],
                "what": "each device's stream from one launch's stop event to the next one's start event (HIP "
                        "events; libnanopow npow_device_stats idle_ms / idle_gaps): with one search per launch, "
                        "the device's idle time per search"},
            "adopt": _mean_p([x.adopt_us for x in infos]),
            "launch_first_device": _mean_p([x.launch_us for x in infos]),
            "launch_last_device": _mean_p([x.launch_all_us or None for x in infos]),
            "win_seen": _mean_p([x.win_seen_us for x in infos]),
            "win_seen_to_decided": _mean_p([x.decide_us - x.win_seen_us for x in infos if x.win_seen_us > 0]),
            "decided_to_result_in_client": _mean_p([r * 1e6 - x.decide_us for r, x in zip(res, infos)]),
            "client_turnaround_to_next_submit": _mean_p(turn),
            "losers_stop_after_decide": _mean_p([x.stop_after_decide_us for x in infos]),
            "collected_after_submit": _mean_p([x.finish_us for x in infos]),
            "what": "host timeline of each search, us since its npow_submit (npow_wait_info, steady clock) -- adopt "
                    "(a device's worker took the job), launch issued on the first / last device, the winning "
                    "device's win record read by the host (the worker's poll: it naps up to 50 us between looks "
                    "once a launch is 0.4 ms old), decided after CPU re-validation, the result in the client's "
                    "thread (Python), the client's turnaround to the next submit, the losing devices' stop as the "
                    "host saw it, the ticket collected (every device stopped)"},
        "launches_per_search_per_device": round(sum(k.launches for k in ks) / (m * n_dev), 3),
        "dyn_entries_per_search_per_device": round(sum(k.dyn_entries for k in ks) / (m * n_dev), 3),
        "late_nonces_losers": _mean_p([x.late_nonces_losers for x in infos]),
        "per_device_kernel_gnps": [round(hash_rate(k) / 1e9, 4) if k.kernel_ms > 0 else None for k in ks],
        "per_device_linger_ms": [round(getattr(k, "linger_ms", 0.0), 2) for k in ks],
        # the worker's 1-ms fallback for a final count that had not come (ABI 6): late ones, and missing ones (0)
        "stale_final_counts": {"stale": sum(getattr(k, "stale_drains", 0) for k in ks),
                               "late": sum(getattr(k, "stale_late", 0) for k in ks),
                               "missing": sum(getattr(k, "stale_missing", 0) for k in ks),
                               "linger_relays": sum(getattr(k, "linger_relays", 0) for k in ks)},
        "in_kernel_mhz": round(statistics.mean([k.clock_mhz for k in ks if k.clock_mhz > 0]), 1)
        if any(k.clock_mhz > 0 for k in ks) else None,
        "worker_core_share": round(sum(k.host_cpu_ms for k in ks) / max(1e-9, ks[0].host_wall_ms), 3),
        "partitions": [[k.hip_device, k.cu_first, k.cus] for k in ks],
    }
    if http_m:
        http = _http_ttw(eng, http_m, thr=thr, base=6_500_000, device_mask=mask)
        line["http_keepalive_ttw_ms"] = {"p50": round(pct(http, 50) * 1e3, 4), "p99": round(pct(http, 99) * 1e3, 4),
                                         "n": len(http),
                                         "hop_p50_ms": round((pct(http, 50) - pct(res, 50)) * 1e3, 4)}
    return line


def workload_regime(eng, args, rank, world, dist):
    """--workload regime: node_regime over --gpus devices of this process (default every visible one)."""
    if world > 1:
        raise SystemExit("--workload regime runs in ONE process (it drives every device itself)")
    n_dev = args.gpus if args.gpus > 1 else eng.n_devices
    thr = int(args.threshold, 16) if args.threshold else REGIME
    reg = node_regime(eng, n_dev, args.steps, thr, http_m=args.http_requests)
    rate = reg["node_gnps"]
    ks = [eng.stats(d) for d in range(n_dev)]
    line = result_line(n_dev, args.steps, 5, int(rate * 1e9), 1.0, [reg["c_abi_ttw_ms"]["p50"] / 1e3],
                       sum(k.kernel_ms for k in ks), sum(k.nonces for k in ks), sum(k.launches for k in ks),
                       parallelism=f"in-process x{n_dev}: one root at a time split over {n_dev} devices, first win "
                                   "cancels the others (no collective)")
    line.pop("max_ttw_ms", None)
    line["unit"] = "Gnonce/s"
    line["scaling"] = "strong"
    line["p50_ttw_ms"], line["p99_ttw_ms"] = reg["c_abi_ttw_ms"]["p50"], reg["c_abi_ttw_ms"]["p99"]
    line["mean_ttw_ms"], line["n_ttw"] = reg["c_abi_ttw_ms"]["mean"], args.steps
    line["roofline"]["kernel_gnps"] = reg["kernel_gnps"]
    line["config"]["workload"] = (f"8-GPU time regime (VERDICT r04 #1): one root at a time at {reg['threshold']} over "
                                  f"{n_dev} devices, the next root submitted at the previous result")
    line["config"]["threshold"] = reg["threshold"]
    line["node_ttw_8x_regime"] = reg
    if os.environ.get("NANOPOW_VIRTUAL_DEVICES"):
        line["virtual_devices_note"] = (f"NANOPOW_VIRTUAL_DEVICES: the {n_dev} devices are CU partitions of one GPU "
                                        "(CU-masked streams), each launch on CUs of its own as on separate GPUs")
    return line


def regime_child(n_dev: int, m: int, timeout: float = 150.0):
    """The 8-GPU time regime on this box as a child process (the device set is fixed at npow_init, process-wide):
    bench.py --workload regime over NANOPOW_VIRTUAL_DEVICES = n_dev CU partitions of GPU 0 when the box has one GPU
    (the rehearsal), or over the first n_dev GPUs when it has that many.  Its node_ttw_8x_regime record, or an
    error record; never fails the bench."""
    import subprocess
    env = dict(os.environ)
    cmd = [sys.executable, os.path.abspath(__file__), "--workload", "regime", "--gpus", str(n_dev), "--steps", str(m),
           "--http-requests", "100"]
    try:
        n_phys = int(subprocess.run([sys.executable, "-c", "import ctypes; h = ctypes.CDLL('libamdhip64.so.7'); "
                                     "n = ctypes.c_int(0); h.hipGetDeviceCount(ctypes.byref(n)); print(n.value)"],
                                    capture_output=True, text=True, timeout=60).stdout.strip() or 0)
    except (OSError, ValueError, subprocess.SubprocessError):
        n_phys = 0
    if n_phys < n_dev:
        env["NANOPOW_VIRTUAL_DEVICES"] = str(n_dev)
    try:
        p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=timeout)
        line = json.loads(p.stdout.strip().splitlines()[-1]) if p.returncode == 0 else None
    except (OSError, ValueError, IndexError, subprocess.SubprocessError) as e:
        return {"error": repr(e)[:300]}
    if line is None:
        return {"error": f"rc {p.returncode}: {p.stderr[-300:]}"}
    rec = line["node_ttw_8x_regime"]
    rec["devices_are"] = (f"{n_dev} CU partitions of GPU 0 (NANOPOW_VIRTUAL_DEVICES, one CU-masked stream each)"
                          if "NANOPOW_VIRTUAL_DEVICES" in env else f"{n_dev} physical GPUs")
    return rec


def workload_receive(eng, args, rank, world, dist):
    """BASELINE configs[0]: work_generate at fffffe0000000000, GPU next to the CPU reference."""
    if world > 1:
        raise SystemExit("--workload receive runs in one process")
    recv = 0xfffffe0000000000
    from nanopow.server import HttpWorkServer, WorkServer
    # GPU through the C ABI
    gpu = []
    for i in range(args.steps):
        dt, _t_all, info = search_to_result(eng, bench_root(20_000_000 + i), recv, bench_start(i), 0)
        gpu.append(dt)
        assert info.status == 0 and info.value >= recv
    # GPU through the HTTP work server (what the DPoW client sees): one keep-alive connection, as
    # the client's aiohttp session, and a new connection per request
    http = _http_ttw(eng, min(args.steps, 300), thr=recv, base=21_000_000, device_mask=0)
    srv = HttpWorkServer(WorkServer(eng, max_active=1), "127.0.0.1", 0).start()
    http_new = []
    try:
        for i in range(min(args.steps, 100)):
            body = json.dumps({"action": "work_generate", "hash": bench_root(23_000_000 + i).hex(),
                               "difficulty": f"{recv:016x}"}).encode()
            t = time.perf_counter()
            cli = KeepAliveClient(srv.address)  # a new connection for this request alone
            try:
                rep = cli.post(json.loads(body))
            finally:
                cli.close()
            http_new.append(time.perf_counter() - t)
            assert "work" in rep
    finally:
        srv.stop()
    # the CPU legs (receive_cpu_legs) ran before the GPU was opened; main() adds them
    line = result_line(1, args.steps, 0, 0, 1.0, gpu, 0.0, 0, 0)
    line.pop("roofline")
    line["value"] = round(pct(gpu, 50) * 1e3, 3)
    line["unit"] = "ms p50 time-to-work (GPU, C ABI)"
    line["higher_is_better"] = False
    line["config"] = {"workload": "BASELINE configs[0]: single work_generate at receive difficulty "
                                  "fffffe0000000000 (expected 2^23 nonces), GPU vs the CPU reference",
                      "threshold": "fffffe0000000000"}
    line["receive"] = {
        "gpu_c_abi_ms": {"p50": round(pct(gpu, 50) * 1e3, 3), "p99": round(pct(gpu, 99) * 1e3, 3), "n": len(gpu)},
        "gpu_http_keepalive_ms": {"p50": round(pct(http, 50) * 1e3, 3), "p99": round(pct(http, 99) * 1e3, 3),
                                  "n": len(http)},
        "gpu_http_new_connection_ms": {"p50": round(pct(http_new, 50) * 1e3, 3),
                                       "p99": round(pct(http_new, 99) * 1e3, 3), "n": len(http_new)},
    }
    return line


def _hashlib_interleaved(job):
    """One process of the all-cores CPU reference search: nonces start + k, start + k + P, ... until a
    value >= thr or another process has found one (the shared flag, checked every 4,096 nonces)."""
    root, thr, start, k, P, limit = job
    b2 = hashlib.blake2b
    flag = _MP_FLAG
    n = (start + k) & ((1 << 64) - 1)
    for c in range(limit):
        if int.from_bytes(b2(n.to_bytes(8, "little") + root, digest_size=8).digest(), "little") >= thr:
            flag.value = 1
            return c + 1, n
        if (c & 4095) == 0 and flag.value:
            return c + 1, None
        n = (n + P) & ((1 << 64) - 1)
    return limit, None


_MP_FLAG = None


def _mp_init(flag):
    global _MP_FLAG
    _MP_FLAG = flag


def receive_cpu_legs(args):
    """BASELINE configs[0]'s CPU side: the reference's CPU path,
    hashlib.blake2b(digest_size=8), on one core and on every granted host core (one process per
    core on interleaved nonces, the first hit ending the request), and the oracle's C port on the
    same cores.  Runs before the GPU is opened (its worker processes are forked)."""
    import multiprocessing
    sys.path.insert(0, os.path.join(HERE, "oracle"))
    import oracle  # CPU baseline legs only
    recv = 0xfffffe0000000000
    cores = granted_cores()
    cpu1, cpu1_nonces = [], 0
    for i in range(args.cpu_requests):
        t = time.perf_counter()
        k, nonce = _hashlib_search(bench_root(22_000_000 + i), recv, bench_start(i), 1 << 28)
        cpu1.append(time.perf_counter() - t)
        cpu1_nonces += k
        assert nonce is not None
    cpun_hl, hl_nonces = [], 0
    ctx = multiprocessing.get_context("fork")
    for i in range(args.cpu_requests):
        root = bench_root(22_000_000 + i)
        flag = ctx.Value("i", 0, lock=False)
        with ctx.Pool(cores, initializer=_mp_init, initargs=(flag,)) as pool:
            t = time.perf_counter()
            parts = pool.map(_hashlib_interleaved, [(root, recv, bench_start(i), k, cores, 1 << 26)
                                                    for k in range(cores)], chunksize=1)
            cpun_hl.append(time.perf_counter() - t)
        found = [n for _, n in parts if n is not None]
        assert found and all(oracle.work_value(root, n) >= recv for n in found)
        hl_nonces += sum(c for c, _ in parts)
    cpun = []
    for i in range(args.cpu_requests):
        root = bench_root(22_000_000 + i)
        t = time.perf_counter()
        oracle.sweep(root, recv, bench_start(i), 1 << 24, threads=cores)  # 2x the expected nonces
        cpun.append(time.perf_counter() - t)
    return {
        "cpu_hashlib_1core_ms": {"p50": round(pct(cpu1, 50) * 1e3, 1), "n": len(cpu1),
                                 "gnps": round(cpu1_nonces / sum(cpu1) / 1e9, 6)},
        "cpu_hashlib_allcores_ms": {"p50": round(pct(cpun_hl, 50) * 1e3, 1), "n": len(cpun_hl), "cores": cores,
                                    "gnps": round(hl_nonces / sum(cpun_hl) / 1e9, 6),
                                    "how": f"hashlib.blake2b in {cores} forked processes on interleaved nonces, the "
                                           "first hit ending the request (pool start-up included)"},
        "cpu_oracle_c_scan_2p24_ms": {"median": round(statistics.median(cpun) * 1e3, 1), "threads": cores,
                                      "gnps": round((1 << 24) / statistics.median(cpun) / 1e9, 5)},
    }


def add_clock(line, clocks, over):
    """The in-kernel shader clock of the timed launches (mean over ranks / devices) and the roofline
    priced at it."""
    if not clocks:
        return
    mhz = statistics.mean(clocks)
    line["sclk_mhz"] = {"mean": round(mhz, 1), over: len(clocks),
                        "source": "in-kernel: s_memtime / s_memrealtime spans of one wave per XCD in every "
                                  f"timed search launch (libnanopow stats clock_mhz), mean over {over}"}
    line["roofline"]["frac_at_measured_sclk"] = round(line["roofline"]["achieved"] / (256 * 128 * mhz * 1e6 / 1e12), 4)
    line["roofline"]["frac_algorithmic_at_measured_sclk"] = round(
        line["roofline"]["achieved_algorithmic"] / (256 * 128 * mhz * 1e6 / 1e12), 4)
    kg = line["roofline"]["kernel_gnps"]
    if kg:  # SIMD cycles per 64-nonce wave-hash at the in-kernel clock (1,024 SIMDs per GPU)
        n = line["n_gpus"]
        line["roofline"]["issue_model"]["kernel_cycles_per_hash"] = round(1024 * 64 * mhz * 1e6 / (kg / n * 1e9), 1)


def main_inprocess(eng, args) -> int:
    """--gpus N > 1 without torch.distributed.run: the product's own multi-GPU path (run_timed_inprocess),
    then one root at a time over all N GPUs (inprocess_node_ttw)."""
    n = args.gpus
    with SclkSampler(0) as sclk:
        nonces, wall, ttw, recs, kern_ms, kern_nonces, launches, ks = run_timed_inprocess(eng, n, args.steps,
                                                                                          args.warmup)
    line = result_line(n, args.steps, args.warmup, nonces, wall, ttw, kern_ms, kern_nonces, launches,
                       parallelism=f"in-process x{n}: the work pool over device_mask = {n} GPUs, {n} searches in "
                                   f"flight, each split into {n} disjoint strides with first-found cancellation "
                                   "(no collective)")
    # kernel_gnps above is per device-second summed over devices: report the node's kernel rate too
    line["roofline"]["kernel_gnps_per_gpu"] = round(kern_nonces / (kern_ms * 1e-3) / 1e9, 4) if kern_ms > 0 else None
    line["roofline"]["kernel_gnps"] = round(kern_nonces / (kern_ms * 1e-3 / n) / 1e9, 4) if kern_ms > 0 else None
    add_clock(line, [k.clock_mhz for k in ks if k.clock_mhz > 0], "devices")
    clk = sclk.summary()
    if clk:
        line["sysfs_sclk_mhz"] = clk
    line["timed_overshoot"] = overshoot_summary([r[2] for r in recs], [r[3] for r in recs], [r[1] for r in recs],
                                                [r[4] for r in recs])
    if os.environ.get("NANOPOW_VIRTUAL_DEVICES"):
        parts = [[k.hip_device, k.cu_first, k.cus] for k in ks]
        if all(p[1] >= 0 for p in parts):
            line["virtual_devices_note"] = (
                f"NANOPOW_VIRTUAL_DEVICES: the {n} devices are CU partitions of one GPU (CU-masked streams, "
                f"[hip device, first CU, CUs] = {parts}): every launch runs from its start on CUs of its own, as on "
                "separate GPUs, but they share one card's clock and power cap and HBM; kernel_gnps_per_gpu is per "
                "partition, the roofline is priced for a whole GPU (a rehearsal of the path)")
        else:
            line["virtual_devices_note"] = (
                f"NANOPOW_VIRTUAL_DEVICES with NANOPOW_VIRTUAL_PARTITION=share: the {n} devices time-share one GPU; "
                "their launches overlap, so per-device kernel times, the roofline and the overshoot spans are not "
                "those of separate GPUs (a rehearsal of the path)")
    line["early_finishes"] = sum(k.early_finishes for k in ks)
    line["kills_relayed"] = sum(k.kills_relayed for k in ks)
    # rates over the time each device hashed: a CU partition that lingered more is not slower
    line["device_check"] = device_check([hash_rate(k) / 1e9 for k in ks], kern_nonces, nonces,
                                        [k.clock_mhz for k in ks])
    if args.node_searches:
        line["node_ttw_ms"] = inprocess_node_ttw(eng, n, args.node_searches)
    print(json.dumps(line), flush=True)
    if not line["device_check"]["ok"]:
        print(f"bench.py: device check failed: {line['device_check']}", file=sys.stderr)
        return 3
    return 0


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1,
                    help="GPUs: under torch.distributed.run it must equal WORLD_SIZE (one rank per GPU); alone, "
                         "N > 1 runs the work pool over N devices in this process")
    ap.add_argument("--steps", type=int, default=300, help="searches per GPU in the timed region")
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--iters", type=int, default=0, help="override the search launch iteration cap")
    ap.add_argument("--budget-us", type=int, default=-1, help="override the search launch budget (0 = off)")
    ap.add_argument("--workload", default="search",
                    choices=["search", "allgpus", "sweep", "burst", "sustained", "dpow", "receive", "regime"])
    ap.add_argument("--threshold", default="", help="regime: threshold in hex (default ffffffc000000000)")
    ap.add_argument("--sweep-bits", type=int, default=36, help="sweep: range [0, 2^bits)")
    ap.add_argument("--roots", type=int, default=4096, help="burst: requests per GPU")
    ap.add_argument("--duration", type=float, default=60.0, help="sustained: seconds")
    ap.add_argument("--depth", type=int, default=4, help="sustained: requests in flight per GPU")
    ap.add_argument("--rate", type=float, default=20.0, help="dpow: work messages per second")
    ap.add_argument("--concurrency", type=int, default=1, help="dpow: WorkHandler loops (reference: 1)")
    ap.add_argument("--cpu-requests", type=int, default=4, help="receive: requests timed on the CPU reference")
    ap.add_argument("--via", choices=["abi", "http"], default="abi",
                    help="burst: submit through the C ABI work pool or POST to the HTTP work server")
    ap.add_argument("--node-searches", type=int, default=300,
                    help="search, N>1: roots searched by all GPUs at once after the timed steps (node time-to-work)")
    ap.add_argument("--http-requests", type=int, default=100,
                    help="search, N=1: work_generate requests timed at the JSON boundary after the timed steps")
    ap.add_argument("--latency-searches", type=int, default=1000,
                    help="search, N=1: C-ABI searches on R_0..R_{n-1} after the timed steps (p50/p99 time-to-work)")
    ap.add_argument("--regime-searches", type=int, default=500,
                    help="search, N=1: searches of the 8-GPU time regime run in a child process after the bench "
                         "(node_ttw_8x_regime; 0 = skip)")
    args = ap.parse_args()
    if args.gpus < 1:
        raise SystemExit("bench.py: --gpus must be >= 1")
    if WORLD > 1 and args.gpus != WORLD:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={WORLD}: under torch.distributed.run "
                         "there is one rank per GPU")
    inproc = WORLD == 1 and args.gpus > 1

    # The CPU legs run first, before anything opens the GPU (their worker processes are forked).
    cpu = None
    if args.workload == "search" and WORLD == 1 and args.gpus == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline()
    recv_cpu = receive_cpu_legs(args) if args.workload == "receive" else None
    if cpu or recv_cpu:
        time.sleep(1.0)  # let the CPU legs' worker processes finish exiting before the GPU work is timed

    rank = int(os.environ.get("RANK", "0"))
    dist = None
    if WORLD > 1:
        import torch.distributed as dist  # gloo: barrier + scalar reductions only
        import datetime
        # a lost rank ends the job within minutes instead of gloo's default 30
        dist.init_process_group("gloo", timeout=datetime.timedelta(seconds=300))

    import nanopow
    from nanopow import _lib
    eng = nanopow.engine()  # fails loudly without libnanopow.so / a GPU: no CPU fallback
    if WORLD > 1 and eng.n_devices != 1 and "NANOPOW_VIRTUAL_DEVICES" not in os.environ:
        raise SystemExit(f"bench.py: rank {rank} sees {eng.n_devices} devices, expected exactly one")
    if eng.n_devices < args.gpus and WORLD == 1:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but only {eng.n_devices} device(s) are visible")
    if args.iters:
        eng.set_tuning(args.iters, 0, 0)
    if args.budget_us >= 0:
        eng.set_pool_tuning(args.budget_us)
    dev = 0  # a rank's only visible GPU; in one process, devices 0..N-1
    if args.workload != "search":
        fn = {"allgpus": workload_allgpus, "sweep": workload_sweep, "burst": workload_burst,
              "sustained": workload_sustained, "dpow": workload_dpow, "receive": workload_receive,
              "regime": workload_regime}[args.workload]
        line = fn(eng, args, rank, WORLD, dist)
        if recv_cpu:
            line["receive"].update(recv_cpu)
        if rank == 0:
            print(json.dumps(line), flush=True)
        if dist is not None:
            dist.barrier()
            dist.destroy_process_group()
        return 0
    if inproc:
        return main_inprocess(eng, args)

    def search(i):
        # time-to-work at the result (npow_wait_result), nonces after the ticket's collection; the timed
        # region's wall time includes the collection (the next search starts after it)
        t_res, _t_all, info = search_to_result(eng, bench_root(i), SEND, bench_start(i), 1 << dev)
        return t_res, info.nonces_done

    timed_stats = []

    def stats():
        st = eng.stats(dev)
        timed_stats.append(st)  # read right after the timed region: its clock and host CPU too
        return st.kernel_ms, st.nonces, st.launches

    with SclkSampler(dev) as sclk:
        res = run_timed(search, stats, lambda: eng.reset_stats(dev), args.steps, args.warmup, rank, WORLD, dist)
    st = timed_stats[-1]
    local = (st.clock_mhz, st.host_cpu_ms / st.host_wall_ms if st.host_wall_ms > 0 else 0.0,
             st.nonces / (st.kernel_ms * 1e-3) / 1e9 if st.kernel_ms > 0 else 0.0)
    if dist is not None:
        gathered = [None] * WORLD
        dist.all_gather_object(gathered, local)
    else:
        gathered = [local]
    kern_rate = res[4] / (res[3] * 1e-3) / 1e9 if res[3] > 0 else None
    lat, lat_clk, steady = None, None, None
    if WORLD == 1 and args.latency_searches:
        # the card's clock and power over the ~11-s time-to-work leg too (the timed region is ~0.2 s at the
        # driver's 20 steps: a handful of samples), every 25 ms, with the in-kernel clock of the same launches
        eng.reset_stats(dev)
        with SclkSampler(dev, period=0.025, span="over the time-to-work leg") as lat_sclk:
            lat = latency_sample(eng, dev, args.latency_searches, kern_rate, snap=lambda: eng.stats(dev))
        leg = lat.pop("_snap")
        lat_clk = {"sysfs_sclk_mhz": lat_sclk.summary(), "sysfs_power_w": lat_sclk.power_summary(),
                   "in_kernel_mhz": round(eng.stats(dev).clock_mhz, 1),
                   "what": f"the {args.latency_searches} time-to-work searches (ttw_c_abi_ms; ~11 s of launches at "
                           "fffffff8 and the receive-difficulty overhead sample) sampled every 25 ms; the in-kernel "
                           "clock of their launches beside"}
        steady = steady_state(lat, leg, lat_sclk, args.latency_searches)
    http = _http_ttw(eng, args.http_requests) if (rank == 0 and WORLD == 1 and args.http_requests) else None
    node = None
    if dist is not None and args.node_searches > 0 and int(os.environ.get("LOCAL_WORLD_SIZE", WORLD)) == WORLD:
        node = node_time_to_work(eng, dev, rank, WORLD, dist, args.node_searches)
    if rank == 0:
        line = result_line(WORLD, args.steps, args.warmup, *res)
        add_clock(line, [g[0] for g in gathered if g[0] > 0], "ranks")
        clk = sclk.summary()
        if clk:
            line["sysfs_sclk_mhz"] = clk
        pw = sclk.power_summary()
        if pw:
            line["sysfs_power_w"] = pw
        line["host_worker_cpu"] = {"max_core_share": round(max(g[1] for g in gathered), 4),
                                   "what": "CPU time of the GPU's pool worker thread / wall time over the timed "
                                           "searches (libnanopow stats host_cpu_ms / host_wall_ms), max over ranks"}
        if lat:
            line["ttw_c_abi_ms"] = lat
        if lat_clk:
            line["ttw_leg_clock_power"] = lat_clk
        if steady:
            line["value_steady"] = steady["value"]
            line["steady_state"] = steady
        if node:
            line["node_ttw_ms"] = node
        if http:
            line["http_ttw_ms"] = {"p50": round(pct(http, 50) * 1e3, 3), "p99": round(pct(http, 99) * 1e3, 3),
                                   "n": len(http), "note": "POST work_generate -> reply over one keep-alive "
                                   "connection to the 127.0.0.1 HTTP work server (as the DPoW client's aiohttp "
                                   "session), after the timed region; not part of value"}
        if cpu:
            line["cpu_baseline"] = cpu
        line["device_check"] = device_check([g[2] for g in gathered], res[4], res[0], [g[0] for g in gathered])
        if WORLD == 1 and args.regime_searches:
            line["node_ttw_8x_regime"] = regime_child(8, args.regime_searches)
        print(json.dumps(line), flush=True)
    rc = 0
    if rank == 0 and not line["device_check"]["ok"]:
        print(f"bench.py: device check failed: {line['device_check']}", file=sys.stderr)
        rc = 3
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()
    return rc


if __name__ == "__main__":
    sys.exit(main())
