#!/usr/bin/env python3
"""Generate the gfx950 instruction stream of the Nano work hash.

Writes ``nano-dpow_amd/csrc/npow_hash_asm.inc``: one inline-asm block that
computes ``value = BLAKE2b-64(LE64(nonce) || root)`` for one nonce per lane,
plus the host function that precomputes every nonce-independent (uniform)
intermediate of it.

Why generate instead of letting hipcc compile the C++ rounds
(npow_kernel.hip's ``work_value_pre``): on gfx950 a 64-bit add is ONE
``v_lshl_add_u64`` (4.4 SIMD cycles, measured in profiles/r01_valu_ubench.json)
but it needs its operands in even-aligned VGPR pairs, while the rotations
produce 32-bit halves (``v_alignbit_b32``).  hipcc's register allocator
reconciles the two with ~330 ``v_mov_b32`` copies per hash and a 233-VGPR
schedule (occupancy 2).  Here the data flow is small and fixed (96 G
functions), so we do the instruction selection, dead-code elimination,
scheduling and register allocation ourselves:

* symbolic evaluation of the 12 rounds: m0 = nonce (per lane), m1..m4 = root
  (uniform), m5..m15 = 0; every node that does not depend on the nonce is
  uniform and moves to the host (``npow_asm_uniforms``) -- this subsumes the
  round-1 column precomputation; only the uniforms the per-lane code reads
  are passed in (as 64-bit SGPR-pair operands);
* dead-code elimination from the single output ``H0 ^ v0 ^ v8`` (round 12's
  unused half disappears);
* instruction selection: add64 -> ``v_lshl_add_u64 d, a, 0, b``;
  rotr32(x ^ y) -> two ``v_xor_b32`` writing swapped halves (the rotation is
  free); rotr{24,16,63}(x ^ y) -> two ``v_xor_b32`` + two ``v_alignbit_b32``;
  xor with a compile-time constant uses a 32-bit literal;
* list scheduling by critical path with a simple latency model;
* linear-scan register allocation at 32-bit granularity with even-aligned
  pairs for 64-bit operands, inside a fixed VGPR window the asm statement
  declares clobbered.

Usage: python3 tools/gen_hash_asm.py [--sched rr|cp|seq] [--base 8] [--check]
``--check`` evaluates the generated instruction stream with a tiny Python
interpreter against hashlib on random inputs before writing the file.
"""
from __future__ import annotations

import argparse
import hashlib
import os
import random
import re
import sys
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

M64 = (1 << 64) - 1
M32 = (1 << 32) - 1

IV = [0x6a09e667f3bcc908, 0xbb67ae8584caa73b, 0x3c6ef372fe94f82b, 0xa54ff53a5f1d36f1,
      0x510e527fade682d1, 0x9b05688c2b3e6c1f, 0x1f83d9abfb41bd6b, 0x5be0cd19137e2179]
H0 = IV[0] ^ 0x01010008
SIGMA = [
    [0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15],
    [14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3],
    [11, 8, 12, 0, 5, 2, 15, 13, 10, 14, 3, 6, 7, 1, 9, 4],
    [7, 9, 3, 1, 13, 12, 11, 14, 2, 6, 5, 10, 4, 0, 15, 8],
    [9, 0, 5, 7, 2, 4, 10, 15, 14, 1, 11, 12, 6, 8, 3, 13],
    [2, 12, 6, 10, 0, 11, 8, 3, 4, 13, 7, 5, 15, 14, 1, 9],
    [12, 5, 1, 15, 14, 13, 4, 10, 0, 7, 6, 3, 9, 2, 8, 11],
    [13, 11, 7, 14, 12, 1, 3, 9, 5, 0, 15, 4, 8, 6, 2, 10],
    [6, 15, 14, 9, 11, 3, 0, 8, 12, 2, 13, 7, 1, 4, 10, 5],
    [10, 2, 8, 4, 7, 6, 1, 5, 15, 11, 9, 14, 3, 12, 13, 0],
    [0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15],
    [14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3],
]


def rotr(x: int, n: int) -> int:
    return ((x >> n) | (x << (64 - n))) & M64


# ---------------------------------------------------------------------------------------
# Symbolic DAG
# kinds: 'nonce', 'root'(i), 'const'(c), 'add'(a,b), 'xor'(a,b), 'rotr'(a,n)
@dataclass(eq=False)
class Node:
    kind: str
    args: tuple = ()
    val: int = 0          # for const
    idx: int = 0          # for root / rotation amount
    uniform: bool = False
    id: int = -1
    g: int = -1           # G-function ordinal (for scheduling tie-breaks)


class Dag:
    def __init__(self) -> None:
        self.nodes: List[Node] = []
        self.cur_g = -1

    def _new(self, n: Node) -> Node:
        n.id = len(self.nodes)
        n.g = self.cur_g
        self.nodes.append(n)
        return n

    def nonce(self) -> Node:
        return self._new(Node("nonce"))

    def root(self, i: int) -> Node:
        return self._new(Node("root", idx=i, uniform=True))

    def const(self, c: int) -> Node:
        return self._new(Node("const", val=c & M64, uniform=True))

    def add(self, a: Node, b: Node) -> Node:
        if a.kind == "const" and b.kind == "const":
            return self.const(a.val + b.val)
        if a.kind == "const" and a.val == 0:
            return b
        if b.kind == "const" and b.val == 0:
            return a
        return self._new(Node("add", (a, b), uniform=a.uniform and b.uniform))

    def xor(self, a: Node, b: Node) -> Node:
        if a.kind == "const" and b.kind == "const":
            return self.const(a.val ^ b.val)
        return self._new(Node("xor", (a, b), uniform=a.uniform and b.uniform))

    def rotr(self, a: Node, n: int) -> Node:
        if a.kind == "const":
            return self.const(rotr(a.val, n))
        return self._new(Node("rotr", (a,), idx=n, uniform=a.uniform))


def build_hash_dag() -> Tuple[Dag, Node]:
    d = Dag()
    zero = d.const(0)
    nonce = d.nonce()
    m = [nonce] + [d.root(i) for i in range(4)] + [zero] * 11
    v = [d.const(x) for x in [H0] + IV[1:8] + IV[0:4] + [IV[4] ^ 40, IV[5], (~IV[6]) & M64, IV[7]]]
    gcount = 0

    def G(a, b, c, dd, x, y):
        nonlocal gcount
        d.cur_g = gcount
        gcount += 1
        v[a] = d.add(d.add(v[a], m[x]), v[b])
        v[dd] = d.rotr(d.xor(v[dd], v[a]), 32)
        v[c] = d.add(v[c], v[dd])
        v[b] = d.rotr(d.xor(v[b], v[c]), 24)
        v[a] = d.add(d.add(v[a], m[y]), v[b])
        v[dd] = d.rotr(d.xor(v[dd], v[a]), 16)
        v[c] = d.add(v[c], v[dd])
        v[b] = d.rotr(d.xor(v[b], v[c]), 63)

    for r in range(12):
        s = SIGMA[r]
        G(0, 4, 8, 12, s[0], s[1])
        G(1, 5, 9, 13, s[2], s[3])
        G(2, 6, 10, 14, s[4], s[5])
        G(3, 7, 11, 15, s[6], s[7])
        G(0, 5, 10, 15, s[8], s[9])
        G(1, 6, 11, 12, s[10], s[11])
        G(2, 7, 8, 13, s[12], s[13])
        G(3, 4, 9, 14, s[14], s[15])
    d.cur_g = gcount
    out = d.xor(d.xor(v[0], v[8]), d.const(H0))
    return d, out


def eval_node(n: Node, nonce: int, root_words: List[int], memo: Dict[int, int]) -> int:
    if n.id in memo:
        return memo[n.id]
    k = n.kind
    if k == "nonce":
        r = nonce
    elif k == "root":
        r = root_words[n.idx]
    elif k == "const":
        r = n.val
    elif k == "add":
        r = (eval_node(n.args[0], nonce, root_words, memo) + eval_node(n.args[1], nonce, root_words, memo)) & M64
    elif k == "xor":
        r = eval_node(n.args[0], nonce, root_words, memo) ^ eval_node(n.args[1], nonce, root_words, memo)
    elif k == "rotr":
        r = rotr(eval_node(n.args[0], nonce, root_words, memo), n.idx)
    else:
        raise ValueError(k)
    memo[n.id] = r
    return r


# ---------------------------------------------------------------------------------------
# Lowering to "ops": each op is a small fixed instruction pattern on 64-bit values.
@dataclass(eq=False)
class Op:
    kind: str               # 'add', 'xrot32', 'xrot', 'xor' (final / plain)
    dst: Node
    srcs: List[Node]        # lane-varying or uniform or const operands
    n: int = 0              # rotation amount
    id: int = -1
    g: int = -1
    users: List["Op"] = field(default_factory=list)
    preds: List["Op"] = field(default_factory=list)
    prio: float = 0.0


def lower(dag: Dag, out: Node):
    """Return (ops in topological order, list of uniform frontier nodes)."""
    # collect live (reachable) lane-varying nodes
    live: Dict[int, Node] = {}
    stack = [out]
    while stack:
        n = stack.pop()
        if n.id in live or n.uniform:
            continue
        live[n.id] = n
        stack.extend(n.args)
    # use counts of xor nodes: an xor feeding only a rotr is fused into it
    users: Dict[int, List[Node]] = {}
    for n in live.values():
        for a in n.args:
            users.setdefault(a.id, []).append(n)
    ops: List[Op] = []
    produced: Dict[int, Op] = {}
    frontier: Dict[int, Node] = {}

    def operand(a: Node, pair: bool = False) -> Node:
        # 64-bit add operands that are uniform (constants included: VOP3 takes no
        # 64-bit literal) come from SGPR pairs; xor takes 32-bit literals directly.
        if a.uniform and (pair or a.kind != "const"):
            frontier[a.id] = a
        return a

    for nid in sorted(live):
        n = live[nid]
        if n.kind == "nonce":
            continue
        if n.kind == "add":
            op = Op("add", n, [operand(n.args[0], True), operand(n.args[1], True)], g=n.g)
        elif n.kind == "rotr":
            x = n.args[0]
            if x.kind == "xor" and not x.uniform and len(users.get(x.id, [])) == 1:
                kind = "xrot32" if n.idx == 32 else "xrot"
                op = Op(kind, n, [operand(x.args[0]), operand(x.args[1])], n=n.idx, g=n.g)
            else:
                raise NotImplementedError("rotation of a non-xor value")
        elif n.kind == "xor":
            us = users.get(n.id, [])
            if us and all(u.kind == "rotr" for u in us) and len(us) == 1:
                continue  # fused into its rotation
            op = Op("xor", n, [operand(n.args[0]), operand(n.args[1])], g=n.g)
        else:
            raise ValueError(n.kind)
        op.id = len(ops)
        ops.append(op)
        produced[n.id] = op
    # dependency edges
    for op in ops:
        for s in op.srcs:
            p = produced.get(s.id)
            if p is not None:
                op.preds.append(p)
                p.users.append(op)
    return ops, list(frontier.values()), produced


# issue cost (SIMD cycles per wave64 instruction, profiles/r01_valu_ubench.json) and latency model
COST = {"v_xor_b32": 2.5, "v_xor_b32_s": 4.7, "v_xor_b32_k": 2.9, "v_alignbit_b32": 4.3, "v_alignbyte_b32": 4.3,
        "v_lshl_add_u64": 4.4,
        "v_lshrrev_b32": 2.5, "v_mov_b32": 2.4, "v_add_co_u32": 2.1, "v_addc_co_u32": 2.1, "v_mad_u32_u24": 4.0,
        "v_bitop3_b32": 2.5}
# 64-bit add as v_add_co_u32 + v_addc_co_u32 (carry through VCC) instead of one v_lshl_add_u64:
# both issue at full rate next to xors (profiles/r01_valu_mix2.jsonl), v_lshl_add_u64 does not
ADD_CC = False
# --add sgpr: the same carry pair in VOP3 form with its carry in an SGPR pair taken round-robin from
# CARRY_SGPRS (v_add_co_u32_e64 v, s[k:k+1], ... / v_addc_co_u32_e64 v, s[k:k+1], ..., s[k:k+1]),
# so consecutive adds do not all write and read VCC
ADD_SGPR = False
CARRY_SGPRS: List[int] = [20, 22, 24, 26]
_carry_turn = [0]


def next_carry() -> str:
    k = CARRY_SGPRS[_carry_turn[0] % len(CARRY_SGPRS)]
    _carry_turn[0] += 1
    return f"s[{k}:{k + 1}]"


ROT_MAD = lambda n, h: False  # which rotr16/24 halves use v_lshrrev_b32 + v_mad_u32_u24 (--rotmad)
ROTL1_CC = False  # rotr63 = x + x + carry as v_add_co_u32 + 2x v_addc_co_u32
ROTL1_VIA_ADD = True  # rotr63 = (x << 1) + (x >> 63): v_lshrrev_b32 + v_lshl_add_u64 with a zero partner
# Measured on MI355X (tools/experiments/valu_patterns.py): in a stream that mixes in 64-bit / 3-operand VALU
# ops, VOP2-encoded v_xor_b32 issues at ~4.1 SIMD cycles but its VOP3 (_e64) encoding at ~2.6.
VOP3_SIMPLE = True
# rotr32 as two in-place xors + two v_mov_b32 into the fresh pair (movs issue nearly free)
SWAP_MOV = False
LAT = 8.0
ZPAIRS = 2  # {t, 0} pairs of the rotl1 trick in use at once (lockstep: one per G of a half-round, +2)
BARRIER_LINES = ["s_barrier"]  # --sched lockstep: what ends an interval (+ "s_nop 0" keeps 8-byte parity)
# --split (lockstep experiments): "order" puts an interval's 64-bit adds (v_lshl_add_u64, the rotl1
# add included) after all its alignbits; "ad" also puts an s_barrier between the two runs; "fh" an
# s_barrier between the full-rate and the half-rate part; "all" both barriers
SPLIT = "none"
ROT_BYTE = False  # --rotbyte (round 3 power experiments): rotr24 / rotr16 halves as v_alignbyte_b32
# --run-order (round 3 power experiments): the order of the ops inside each run of a lockstep interval --
# "id" (program order), "rev" (reverse), "shufN" (seeded shuffle); dependencies inside a run still hold
RUN_ORDER = "id"


def order_runs(units, ops_by_id):
    """Reorder the units of each (interval, part) run per RUN_ORDER, topologically (Kahn)."""
    if RUN_ORDER == "id":
        return units
    import heapq
    import random
    rng = random.Random(int(RUN_ORDER[4:]) if RUN_ORDER.startswith("shuf") else 0)
    out, i = [], 0
    while i < len(units):
        j = i
        while j < len(units) and units[j][1] == units[i][1]:
            j += 1
        grp = units[i:j]
        ids = {u[0][0] for u in grp}
        rank = {u[0][0]: (-u[0][0] if RUN_ORDER == "rev" else rng.random()) for u in grp}
        deps = {u[0][0]: {p.id for p in ops_by_id[u[0][0]].preds if p.id in ids} for u in grp}
        by_id = {u[0][0]: u for u in grp}
        indeg = {k: len(v) for k, v in deps.items()}
        users = {k: [m for m in ids if k in deps[m]] for k in ids}
        heap = [(rank[k], k) for k in ids if indeg[k] == 0]
        heapq.heapify(heap)
        while heap:
            _, k = heapq.heappop(heap)
            out.append(by_id[k])
            for m in users[k]:
                indeg[m] -= 1
                if indeg[m] == 0:
                    heapq.heappush(heap, (rank[m], m))
        assert len(out) == j, "cycle inside a run"
        i = j
    return out


def op_cost(op: Op) -> float:
    def xc(s):
        if s.kind == "const":
            return COST["v_xor_b32_k"]
        if s.uniform:
            return COST["v_xor_b32_s"]
        return COST["v_xor_b32"]
    if op.kind == "add":
        return COST["v_lshl_add_u64"]
    x = 2 * max(xc(op.srcs[0]), xc(op.srcs[1]))
    if op.kind == "xrot" and op.n == 63 and ROTL1_VIA_ADD:
        return x + COST["v_lshrrev_b32"] + COST["v_lshl_add_u64"]
    if op.kind == "xrot":
        return x + 2 * COST["v_alignbit_b32"]
    return x


def schedule(ops: List[Op], mode: str) -> List[Op]:
    # priority = longest path (in cost) to the end
    for op in reversed(ops):
        op.prio = op_cost(op) + LAT + max((u.prio for u in op.users), default=0.0)
    if mode == "seq":
        return list(ops)
    n_pred = {op.id: len(op.preds) for op in ops}
    ready_at = {op.id: 0.0 for op in ops}
    ready = [op for op in ops if not op.preds]
    t = 0.0
    order: List[Op] = []
    last_g = -1
    while ready:
        avail = [op for op in ready if ready_at[op.id] <= t]
        pool = avail if avail else ready
        if mode == "cp":
            best = max(pool, key=lambda o: (o.prio, -o.id))
        elif mode == "rr":
            # round-robin over G functions among available ops, preferring a different G than last
            cand = [o for o in pool if o.g != last_g] or pool
            best = max(cand, key=lambda o: (o.prio, -o.id))
        else:
            raise ValueError(mode)
        ready.remove(best)
        if not avail:
            t = ready_at[best.id]
        t += op_cost(best)
        last_g = best.g
        order.append(best)
        for u in best.users:
            n_pred[u.id] -= 1
            ready_at[u.id] = max(ready_at[u.id], t + LAT)
            if n_pred[u.id] == 0:
                ready.append(u)
    assert len(order) == len(ops)
    return order


def schedule_lockstep(ops: List[Op], shift: bool = False, pad_end: bool = False) -> list:
    """--sched lockstep: the 4 independent G functions of each half-round advance together through
    intervals, each interval = the full-rate part of one G step for all of them (xors, the rotl1
    shift) followed by the half-rate part of the next (64-bit adds, alignbits, the rotl1 add), and
    an s_barrier ends every interval.  In a workgroup of 4 waves per SIMD the barrier keeps the
    SIMD's waves in the same phase (tools/experiments/phase_lockstep.py: hash-shaped intervals cost
    ~3.0 cycles per instruction with barriers, 3.7 without).  Returns items for emit(): ops, (op,
    "F") / (op, "H") halves of a split rotation, and "BARRIER".

    shift: the anti-phase stream -- every interval's half-rate part moves to the front of the next
    interval, so an interval is (H of step i-1, F of step i): run beside the unshifted stream on the
    other waves of a SIMD, full-rate and half-rate runs overlap.  It has one more interval than the
    unshifted stream; pad_end gives the unshifted one a trailing barrier so the counts match."""
    by_g: Dict[int, List[Op]] = {}
    for op in ops:
        by_g.setdefault(op.g, []).append(op)
    key: Dict[Tuple[int, str], Tuple[int, int]] = {}   # (op id, part) -> (interval, 0 = F / 1 = H)
    dph = 2 if SPLIT != "none" else 1  # the adds' part: after the alignbits with --split
    assert not (shift and dph == 2), "--shift and --split do not combine"
    for g, gops in by_g.items():
        L = 0
        base = 4 * (g // 4)  # 4 intervals per half-round
        for op in gops:
            if op.kind == "add":
                key[(op.id, "all")] = (base + L, dph)
            elif op.kind == "xrot32":
                L += 1
                key[(op.id, "all")] = (base + L, 0)
            elif op.kind == "xrot":
                L += 1
                key[(op.id, "F")] = (base + L, 0)
                key[(op.id, "H")] = (base + L, dph if (op.n == 63 and ROTL1_VIA_ADD) else 1)
            else:  # the output xor
                key[(op.id, "all")] = (base + L + 1, 0)
    # dependencies win over the pattern: an op is never placed before what it reads
    done: Dict[int, Tuple[int, int]] = {}
    for op in ops:  # topological
        parts = ["F", "H"] if (op.id, "F") in key else ["all"]
        lo = max((done[p.id] for p in op.preds), default=(0, 0))
        prev = lo
        for part in parts:
            k = max(key[(op.id, part)], prev)
            key[(op.id, part)] = k
            prev = k
        done[op.id] = prev
    if shift:  # (iv, F) -> (iv, 2nd); (iv, H) -> (iv + 1, 1st): monotone, so dependencies still hold
        key = {k: (iv + ph, 1 - ph) for k, (iv, ph) in key.items()}
    units = sorted(key.items(), key=lambda kv: (kv[1][0], kv[1][1], kv[0][0]))
    idx = {op.id: op for op in ops}
    units = order_runs(units, idx)
    items: list = []
    cur = None
    cur_ph = 0
    for (oid, part), (iv, ph) in units:
        if cur is not None and iv != cur:
            items.append("BARRIER")
        elif cur is not None and ph != cur_ph and (
                (SPLIT in ("fh", "all") and cur_ph == 0) or (SPLIT in ("ad", "all") and cur_ph == 1 and ph == 2)):
            items.append("BARRIER")
        cur, cur_ph = iv, ph
        items.append((idx[oid], part) if part != "all" else idx[oid])
    if pad_end:
        items.append("BARRIER")
    return items


# ---------------------------------------------------------------------------------------
# Register allocation + emission
# --alloc (round 3 power experiments): which free VGPR the allocator takes -- the lowest (low), the
# highest (high), or the next one after the last taken, wrapping (rr)
ALLOC = "low"


class Alloc:
    def __init__(self, base: int, limit: int) -> None:
        self.base, self.limit = base, limit
        self.free = set(range(base, limit))
        self.max_used = base
        self.last = base - 1

    def _order(self):
        f = sorted(self.free)
        if ALLOC == "high":
            return f[::-1]
        if ALLOC == "rr":
            k = next((i for i, r in enumerate(f) if r > self.last), 0)
            return f[k:] + f[:k]
        return f

    def take1(self, avoid=()) -> int:
        for r in self._order():
            if r not in avoid:
                self.free.remove(r)
                self.max_used = max(self.max_used, r + 1)
                self.last = r
                return r
        raise RuntimeError("out of VGPRs")

    def take2(self, avoid=()) -> int:
        for r in self._order():
            if r % 2 == 0 and r + 1 in self.free and r not in avoid and r + 1 not in avoid:
                self.last = r + 1
                self.free.remove(r)
                self.free.remove(r + 1)
                self.max_used = max(self.max_used, r + 2)
                return r
        raise RuntimeError("out of VGPR pairs")

    def release(self, r: int) -> None:
        assert r not in self.free
        self.free.add(r)


def emit(order: List[Op], frontier: List[Node], out: Node, base: int, limit: int):
    """Return (asm lines, uniform operand index map, max vgpr used, counts)."""
    uni_index = {n.id: i for i, n in enumerate(frontier)}
    # remaining-use counters per lane-varying node (64-bit), counting each op read once
    remaining: Dict[int, int] = {}
    for item in order:
        if isinstance(item, str) or (isinstance(item, tuple) and item[1] == "H"):
            continue  # barriers; a split op's sources are read by its F part
        op = item[0] if isinstance(item, tuple) else item
        for s in op.srcs:
            if not s.uniform:
                remaining[s.id] = remaining.get(s.id, 0) + 1
    al = Alloc(base, limit)
    loc: Dict[int, int] = {}  # node id -> even base register of its pair
    # {t, 0} pairs for rotr63 = (x << 1) + (x >> 63): the odd register of each holds zero
    zpairs = []
    lines_pre: List[str] = []
    if ROTL1_VIA_ADD and not ROTL1_CC:
        for _ in range(ZPAIRS):
            r = al.take2()
            zpairs.append(r)
            lines_pre.append(f"v_mov_b32 v{r + 1}, 0")
    zturn = [0]
    NONCE = "%[nonce]"
    lines: List[str] = []
    counts: Dict[str, int] = {}

    def cnt(k):
        counts[k] = counts.get(k, 0) + 1

    def pair(n: Node) -> str:
        if n.kind == "nonce":
            return NONCE
        if n.uniform:
            return f"%[u{uni_index[n.id]}]"
        r = loc[n.id]
        return f"v[{r}:{r + 1}]"

    def half(n: Node, hi: int) -> str:
        """32-bit operand text for half `hi` of n (for v_xor_b32 src0 may be literal or SGPR)."""
        if n.kind == "const":
            return f"0x{(n.val >> (32 * hi)) & M32:08x}"
        if n.kind == "nonce":
            return f"%[nonce_{'hi' if hi else 'lo'}]"
        if n.uniform:
            return f"%[u{uni_index[n.id]}_{'hi' if hi else 'lo'}]"
        return f"v{loc[n.id] + hi}"

    def dying(op: Op) -> List[Node]:
        ds = []
        seen = set()
        for s in op.srcs:
            if s.uniform or s.kind == "nonce" or s.id in seen:
                continue
            seen.add(s.id)
            if remaining[s.id] == sum(1 for x in op.srcs if x.id == s.id):
                ds.append(s)
        return ds

    def consume(op: Op) -> None:
        seen = set()
        for s in op.srcs:
            if s.uniform or s.kind == "nonce" or s.id in seen:
                continue
            seen.add(s.id)
            remaining[s.id] -= sum(1 for x in op.srcs if x.id == s.id)
            if remaining[s.id] == 0:
                r = loc.pop(s.id)
                al.release(r)
                al.release(r + 1)

    def xor_operands(a: Node, b: Node, hi: int) -> Tuple[str, str]:
        # VOP2 v_xor_b32: src0 may be VGPR/SGPR/literal, src1 must be VGPR
        if not (a.uniform or a.kind == "nonce") or (b.kind == "const" or b.uniform):
            a, b = b, a
        if (a.uniform or a.kind == "const") and (b.uniform or b.kind == "const"):
            raise RuntimeError("uniform xor uniform should have been folded")
        # b must be in a VGPR: nonce or lane-varying
        return half(a, hi), half(b, hi)

    pend: Dict[int, Tuple[int, int]] = {}  # split xrot ops (--sched lockstep): temps between F and H parts
    for item in order:
        if isinstance(item, str):  # "BARRIER": the end of a lockstep interval
            lines.extend(BARRIER_LINES)
            continue
        op, part = item if isinstance(item, tuple) else (item, "all")
        a, b = op.srcs
        if op.kind == "add":
            if a.uniform and b.uniform:
                raise RuntimeError("uniform add should have been folded")
            # one instruction reads both sources before writing: in place on a dying source is fine
            ta, tb = pair(a), pair(b)
            if a.uniform:  # VOP3 src0 may be an SGPR pair too, keep the VGPR first for readability
                ta, tb = tb, ta
            # VOP2 co/addc: src1 must be a VGPR, src0 may be an SGPR; v{r} (even) never aliases a hi half
            x, y = (b, a) if a.uniform else (a, b)
            if y.uniform:
                x, y = y, x
            # v_addc reads VCC over the constant bus, which gfx950 allows only one read per
            # instruction: an add with an SGPR/literal operand stays one v_lshl_add_u64
            cc = (ADD_CC or ADD_SGPR) and not (a.uniform or b.uniform)
            hx = [half(x, 0), half(x, 1)] if cc else None
            hy = [half(y, 0), half(y, 1)] if cc else None
            consume(op)
            r = al.take2()
            loc[op.dst.id] = r
            if cc and ADD_SGPR:
                c = next_carry()
                lines.append(f"v_add_co_u32_e64 v{r}, {c}, {hx[0]}, {hy[0]}")
                lines.append(f"v_addc_co_u32_e64 v{r + 1}, {c}, {hx[1]}, {hy[1]}, {c}")
                cnt("v_add_co_u32")
                cnt("v_addc_co_u32")
            elif cc:
                lines.append(f"v_add_co_u32 v{r}, vcc, {hx[0]}, {hy[0]}")
                lines.append(f"v_addc_co_u32 v{r + 1}, vcc, {hx[1]}, {hy[1]}, vcc")
                cnt("v_add_co_u32")
                cnt("v_addc_co_u32")
            else:
                lines.append(f"v_lshl_add_u64 v[{r}:{r + 1}], {ta}, 0, {tb}")
                cnt("v_lshl_add_u64")
        elif op.kind == "xrot32" and SWAP_MOV:
            s0h, s1h = xor_operands(a, b, 1)
            s0l, s1l = xor_operands(a, b, 0)
            consume(op)
            tl = al.take1()
            th = al.take1(avoid=(tl,))
            lines.append(f"v_xor_b32 v{tl}, {s0l}, {s1l}")
            lines.append(f"v_xor_b32 v{th}, {s0h}, {s1h}")
            r = al.take2(avoid=(tl, th))
            loc[op.dst.id] = r
            lines.append(f"v_mov_b32 v{r}, v{th}")
            lines.append(f"v_mov_b32 v{r + 1}, v{tl}")
            al.release(tl)
            al.release(th)
            cnt("v_xor_b32")
            cnt("v_xor_b32")
            cnt("v_mov_b32")
            cnt("v_mov_b32")
        elif op.kind == "xrot32":
            # dst.lo = a.hi ^ b.hi ; dst.hi = a.lo ^ b.lo  (rotation by 32 is the swap).
            # dst.lo is written before the lo halves are read: keep it off them.
            s0h, s1h = xor_operands(a, b, 1)
            s0l, s1l = xor_operands(a, b, 0)
            lo_regs = tuple(loc[x.id] for x in (a, b) if x.id in loc)
            consume(op)
            r = al.take2(avoid=lo_regs)
            loc[op.dst.id] = r
            lines.append(f"v_xor_b32 v{r}, {s0h}, {s1h}")
            lines.append(f"v_xor_b32 v{r + 1}, {s0l}, {s1l}")
            cnt("v_xor_b32")
            cnt("v_xor_b32")
        elif op.kind == "xrot" and op.n == 63 and ROTL1_CC:
            # rotl1(x) = x + x + (x >> 63): lo+lo carries lo's top bit into hi+hi, whose own carry-out
            # (hi's top bit) is added back into the (even) low word
            s0l, s1l = xor_operands(a, b, 0)
            s0h, s1h = xor_operands(a, b, 1)
            consume(op)
            r = al.take2()
            lines.append(f"v_xor_b32 v{r}, {s0l}, {s1l}")
            lines.append(f"v_xor_b32 v{r + 1}, {s0h}, {s1h}")
            if ADD_SGPR:
                c = next_carry()
                lines.append(f"v_add_co_u32_e64 v{r}, {c}, v{r}, v{r}")
                lines.append(f"v_addc_co_u32_e64 v{r + 1}, {c}, v{r + 1}, v{r + 1}, {c}")
                lines.append(f"v_addc_co_u32_e64 v{r}, {c}, 0, v{r}, {c}")
            else:
                lines.append(f"v_add_co_u32 v{r}, vcc, v{r}, v{r}")
                lines.append(f"v_addc_co_u32 v{r + 1}, vcc, v{r + 1}, v{r + 1}, vcc")
                lines.append(f"v_addc_co_u32 v{r}, vcc, 0, v{r}, vcc")
            loc[op.dst.id] = r
            cnt("v_xor_b32")
            cnt("v_xor_b32")
            cnt("v_add_co_u32")
            cnt("v_addc_co_u32")
            cnt("v_addc_co_u32")
        elif op.kind == "xrot" and op.n == 63 and ROTL1_VIA_ADD:
            if part == "H":  # second half of a split op: x << 1 + {x >> 63, 0}
                r, z = pend.pop(op.id)
                lines.append(f"v_lshl_add_u64 v[{r}:{r + 1}], v[{r}:{r + 1}], 1, v[{z}:{z + 1}]")
                cnt("v_lshl_add_u64")
                continue
            s0l, s1l = xor_operands(a, b, 0)
            s0h, s1h = xor_operands(a, b, 1)
            consume(op)
            r = al.take2()  # x = a ^ b: lo written first (hi sources are odd registers, never r)
            lines.append(f"v_xor_b32 v{r}, {s0l}, {s1l}")
            lines.append(f"v_xor_b32 v{r + 1}, {s0h}, {s1h}")
            z = zpairs[zturn[0] % len(zpairs)]
            zturn[0] += 1
            lines.append(f"v_lshrrev_b32 v{z}, 31, v{r + 1}")
            loc[op.dst.id] = r
            cnt("v_xor_b32")
            cnt("v_xor_b32")
            cnt("v_lshrrev_b32")
            if part == "F":
                pend[op.id] = (r, z)
                continue
            lines.append(f"v_lshl_add_u64 v[{r}:{r + 1}], v[{r}:{r + 1}], 1, v[{z}:{z + 1}]")
            cnt("v_lshl_add_u64")
        elif op.kind == "xrot":
            if part == "H":
                tl, th = pend.pop(op.id)
            else:
                s0l, s1l = xor_operands(a, b, 0)
                s0h, s1h = xor_operands(a, b, 1)
                hi_regs = tuple(loc[x.id] + 1 for x in (a, b) if x.id in loc)
                consume(op)
                tl = al.take1(avoid=hi_regs)   # written before the hi halves are read
                th = al.take1(avoid=(tl,))
                lines.append(f"v_xor_b32 v{tl}, {s0l}, {s1l}")
                lines.append(f"v_xor_b32 v{th}, {s0h}, {s1h}")
                cnt("v_xor_b32")
                cnt("v_xor_b32")
                if part == "F":
                    pend[op.id] = (tl, th)
                    continue
            r = al.take2(avoid=(tl, th))
            loc[op.dst.id] = r
            n = op.n
            # half h of rotr_n: (x_h >> n) | (x_other << (32 - n)) -- one v_alignbit_b32, or
            # v_lshrrev_b32 + v_mad_u32_u24 (x_other[23:0] * 2^(32-n) + (x_h >> n); exact for
            # n = 16, 24), which runs in the multiplier next to alignbit / v_lshl_add_u64
            for h, (xa, xb) in enumerate(((tl, th), (th, tl))):
                if n < 32 and n in (16, 24) and ROT_MAD(n, h):
                    lines.append(f"v_lshrrev_b32 v{r + h}, {n}, v{xa}")
                    lines.append(f"v_mad_u32_u24 v{r + h}, v{xb}, %[k{32 - n}], v{r + h}")
                    cnt("v_lshrrev_b32")
                    cnt("v_mad_u32_u24")
                elif n < 32 and ROT_BYTE:  # --rotbyte: the byte-granular funnel shift (same class)
                    lines.append(f"v_alignbyte_b32 v{r + h}, v{xb}, v{xa}, {n // 8}")
                    cnt("v_alignbyte_b32")
                elif n < 32:
                    lines.append(f"v_alignbit_b32 v{r + h}, v{xb}, v{xa}, {n}")
                    cnt("v_alignbit_b32")
                else:
                    lines.append(f"v_alignbit_b32 v{r + h}, v{xa}, v{xb}, {n - 32}")
                    cnt("v_alignbit_b32")
            al.release(tl)
            al.release(th)
        elif op.kind == "xor":
            s0l, s1l = xor_operands(a, b, 0)
            s0h, s1h = xor_operands(a, b, 1)
            consume(op)
            if op.dst is out:
                lines.append(f"v_xor_b32 %[value_lo], {s0l}, {s1l}")
                lines.append(f"v_xor_b32 %[value_hi], {s0h}, {s1h}")
            else:
                r = al.take2()
                loc[op.dst.id] = r
                lines.append(f"v_xor_b32 v{r}, {s0l}, {s1l}")
                lines.append(f"v_xor_b32 v{r + 1}, {s0h}, {s1h}")
            cnt("v_xor_b32")
            cnt("v_xor_b32")
        else:
            raise ValueError(op.kind)
    for ln in lines_pre:
        cnt(ln.split(" ", 1)[0])
    out_lines = lines_pre + lines
    if VOP3_SIMPLE:
        conv = []
        for ln in out_lines:
            if " " not in ln:  # s_barrier
                conv.append(ln)
                continue
            opc, rest = ln.split(" ", 1)
            if opc in ("v_xor_b32", "v_lshrrev_b32") and "0x" not in rest:
                opc += "_e64"
            conv.append(f"{opc} {rest}")
        out_lines = conv
    return out_lines, uni_index, al.max_used, counts



# ---------------------------------------------------------------------------------------
# Instruction-level backend: lower ops to single instructions on virtual registers, list-schedule
# them with a per-instruction issue cost + result latency model (window-limited to bound register
# pressure), then allocate physical VGPRs (even-aligned pairs for 64-bit operands).
class VR:
    __slots__ = ("id", "pair", "phys")

    def __init__(self, i: int, pair: bool) -> None:
        self.id, self.pair, self.phys = i, pair, None


class Ins:
    __slots__ = ("opc", "dst", "srcs", "imm", "id", "preds", "succs", "prio", "seq", "vop2")

    def __init__(self, opc, dst, srcs, imm=None, vop2=False):
        self.opc, self.dst, self.srcs, self.imm, self.vop2 = opc, dst, srcs, imm, vop2
        self.preds, self.succs = [], []
        self.prio = 0.0


ICOST = {"v_xor_b32": 2.6, "v_xor_b32_k": 2.9, "v_xor_b32_s": 4.7, "v_alignbit_b32": 4.2, "v_lshl_add_u64": 4.35}


def lower_ilp(ops: List[Op], frontier: List[Node], out: Node):
    uni_index = {n.id: i for i, n in enumerate(frontier)}
    vrs: List[VR] = []
    node_vr: Dict[int, VR] = {}
    ins: List[Ins] = []

    def newvr(pair):
        v = VR(len(vrs), pair)
        vrs.append(v)
        return v

    def opnd(n: Node, half):
        """half None = 64-bit operand."""
        if n.kind == "nonce":
            return ("nonce", half)
        if n.uniform:
            if half is not None and n.kind == "const":
                return ("lit", (n.val >> (32 * half)) & M32)
            return ("uni", uni_index[n.id], half)
        return ("vr", node_vr[n.id], half)

    def xor_pair(a: Node, b: Node, half: int):
        sa, sb = opnd(a, half), opnd(b, half)
        # VOP2 needs the literal / SGPR in src0; VOP3 (e64) takes one SGPR anywhere and no literal
        if sb[0] in ("lit", "uni") or (sa[0] == "vr" and sb[0] == "nonce"):
            sa, sb = sb, sa
        return [sa, sb], sa[0] == "lit"

    for op in ops:
        a, b = op.srcs
        if op.kind == "add":
            d = newvr(True)
            node_vr[op.dst.id] = d
            sa, sb = opnd(a, None), opnd(b, None)
            if sa[0] != "vr" and sb[0] == "vr":
                sa, sb = sb, sa
            ins.append(Ins("v_lshl_add_u64", (d, None), [sa, sb]))
        elif op.kind == "xrot32":
            d = newvr(True)
            node_vr[op.dst.id] = d
            for h in (0, 1):
                srcs, lit = xor_pair(a, b, 1 - h)
                ins.append(Ins("v_xor_b32", (d, h), srcs, vop2=lit))
        elif op.kind == "xrot":
            tl, th = newvr(False), newvr(False)
            for t, h in ((tl, 0), (th, 1)):
                srcs, lit = xor_pair(a, b, h)
                ins.append(Ins("v_xor_b32", (t, None), srcs, vop2=lit))
            d = newvr(True)
            node_vr[op.dst.id] = d
            n = op.n
            if n < 32:
                ins.append(Ins("v_alignbit_b32", (d, 0), [("vr", th, None), ("vr", tl, None)], imm=n))
                ins.append(Ins("v_alignbit_b32", (d, 1), [("vr", tl, None), ("vr", th, None)], imm=n))
            else:
                ins.append(Ins("v_alignbit_b32", (d, 0), [("vr", tl, None), ("vr", th, None)], imm=n - 32))
                ins.append(Ins("v_alignbit_b32", (d, 1), [("vr", th, None), ("vr", tl, None)], imm=n - 32))
        elif op.kind == "xor":
            if op.dst is out:
                d = "out"
            else:
                d = newvr(True)
                node_vr[op.dst.id] = d
            for h in (0, 1):
                srcs, lit = xor_pair(a, b, h)
                ins.append(Ins("v_xor_b32", (d, h), srcs, vop2=lit))
        else:
            raise NotImplementedError(op.kind)
    for i, x in enumerate(ins):
        x.id = i
    # dependencies (RAW) at half granularity
    writer: Dict[Tuple[int, int], Ins] = {}
    for x in ins:
        for s in x.srcs:
            if s[0] != "vr":
                continue
            v, half = s[1], s[2]
            keys = [(v.id, 0), (v.id, 1)] if (v.pair and half is None) else [(v.id, half if v.pair else 0)]
            for k in keys:
                w = writer.get(k)
                if w is not None and w not in x.preds:
                    x.preds.append(w)
                    w.succs.append(x)
        d, h = x.dst
        if d != "out":
            if d.pair and h is None:
                writer[(d.id, 0)] = x
                writer[(d.id, 1)] = x
            else:
                writer[(d.id, h if d.pair else 0)] = x
    return ins, vrs


def icost(x: Ins) -> float:
    if x.opc == "v_xor_b32":
        if any(s[0] == "lit" for s in x.srcs):
            return ICOST["v_xor_b32_k"]
        if any(s[0] == "uni" for s in x.srcs):
            return ICOST["v_xor_b32_s"]
    return ICOST[x.opc]


def schedule_ilp(ins: List[Ins], lat: float, window: int) -> List[Ins]:
    for x in reversed(ins):
        x.prio = icost(x) + lat + max((u.prio for u in x.succs), default=0.0)
    npred = {x.id: len(x.preds) for x in ins}
    ready_at = {x.id: 0.0 for x in ins}
    done = [False] * len(ins)
    ready = set(x.id for x in ins if not x.preds)
    first_open = 0
    t = 0.0
    order = []
    while len(order) < len(ins):
        while done[first_open]:
            first_open += 1
        lim = first_open + window
        cand = [ins[i] for i in ready if i < lim]
        avail = [x for x in cand if ready_at[x.id] <= t]
        pool = avail or cand
        if not pool:
            raise RuntimeError("scheduler stuck")
        best = max(pool, key=lambda x: (x.prio, -x.id))
        if not avail:
            t = ready_at[best.id]
        ready.discard(best.id)
        done[best.id] = True
        t += icost(best)
        order.append(best)
        for u in best.succs:
            npred[u.id] -= 1
            ready_at[u.id] = max(ready_at[u.id], t + lat)
            if npred[u.id] == 0:
                ready.add(u.id)
    return order


def allocate_and_emit(order: List[Ins], vrs: List[VR], base: int, limit: int, vop3: bool):
    last_use: Dict[int, int] = {}
    for i, x in enumerate(order):
        for s in x.srcs:
            if s[0] == "vr":
                last_use[s[1].id] = i
    al = Alloc(base, limit)
    lines: List[str] = []
    counts: Dict[str, int] = {}

    def txt(s, pairwise=False):
        k = s[0]
        if k == "lit":
            return f"0x{s[1]:08x}"
        if k == "nonce":
            return "%[nonce]" if s[1] is None else f"%[nonce_{'hi' if s[1] else 'lo'}]"
        if k == "uni":
            return f"%[u{s[1]}]" if s[2] is None else f"%[u{s[1]}_{'hi' if s[2] else 'lo'}]"
        v, half = s[1], s[2]
        if v.pair:
            if half is None:
                return f"v[{v.phys}:{v.phys + 1}]"
            return f"v{v.phys + half}"
        return f"v{v.phys}"

    for i, x in enumerate(order):
        srcs_txt = [txt(s) for s in x.srcs]
        dying = [s[1] for s in x.srcs if s[0] == "vr" and last_use[s[1].id] == i]
        dying = list({v.id: v for v in dying}.values())
        d, h = x.dst
        whole = d != "out" and (not d.pair or h is None)
        if d != "out" and d.phys is None:
            if whole:  # one instruction writes all of d: it may reuse a source dying here
                for v in dying:
                    al.release(v.phys)
                    if v.pair:
                        al.release(v.phys + 1)
                d.phys = al.take2() if d.pair else al.take1()
                for v in dying:
                    for r in ([v.phys, v.phys + 1] if v.pair else [v.phys]):
                        if r != d.phys and not (d.pair and r == d.phys + 1):
                            al.free.discard(r)  # back to allocated state, freed below
                dying_done = True
            else:
                d.phys = al.take2()
                dying_done = False
        else:
            dying_done = False
        if d == "out":
            dtxt = f"%[value_{'hi' if h else 'lo'}]"
        elif d.pair:
            dtxt = f"v[{d.phys}:{d.phys + 1}]" if h is None else f"v{d.phys + h}"
        else:
            dtxt = f"v{d.phys}"
        opc = x.opc
        if opc == "v_lshl_add_u64":
            line = f"{opc} {dtxt}, {srcs_txt[0]}, 0, {srcs_txt[1]}"
        elif opc == "v_alignbit_b32":
            line = f"{opc} {dtxt}, {srcs_txt[0]}, {srcs_txt[1]}, {x.imm}"
        else:
            e = "" if (x.vop2 or not vop3) else "_e64"
            line = f"{opc}{e} {dtxt}, {srcs_txt[0]}, {srcs_txt[1]}"
        lines.append(line)
        counts[opc] = counts.get(opc, 0) + 1
        # free everything whose last use was this instruction (unless it now holds d)
        for v in dying:
            regs = [v.phys, v.phys + 1] if v.pair else [v.phys]
            for r in regs:
                if d != "out" and d.phys is not None and (r == d.phys or (d.pair and r == d.phys + 1)):
                    continue
                if r not in al.free:
                    al.release(r)
    return lines, al.max_used, counts

# ---------------------------------------------------------------------------------------
# A tiny interpreter of the emitted text, to check the generator itself against hashlib.
def fuse_output_xor(lines: List[str], counts: Dict[str, int]) -> List[str]:
    """value = H0 ^ (v0 ^ v8): the stream ends, per half, in `v_xor_b32_e64 t, a, b` and
    `v_xor_b32 %[value_*], <H0 literal>, t`.  Fold each pair into one 3-input
    `v_bitop3_b32 %[value_*], a, b, %[h0_*] bitop3:0x96` (x ^ y ^ z) with the H0 half in an SGPR
    (VOP3 takes no literal on gfx950): 2 instructions fewer per nonce.  Applied only where t is
    read by nothing else and a, b are not rewritten between t's definition and the output."""
    out = list(lines)

    def dst(ln):
        return ln.split(" ", 1)[1].split(",")[0].strip() if " " in ln else ""

    def srcs(ln):
        return [t.strip().split(" ")[0] for t in ln.split(" ", 1)[1].split(",")[1:]] if " " in ln else []

    for half, name in ((0, "value_lo"), (1, "value_hi")):
        k = next((i for i, ln in enumerate(out) if ln.startswith("v_xor_b32 ") and dst(ln) == f"%[{name}]"), None)
        if k is None:
            continue
        lit, t = srcs(out[k])
        if not (lit.startswith("0x") and int(lit, 16) == (H0 >> (32 * half)) & M32 and t.startswith("v")):
            continue
        d = max((i for i in range(k) if dst(out[i]) == t or dst(out[i]).startswith("v[")
                 and t in _pair_regs(dst(out[i]))), default=None)
        if d is None or not out[d].startswith("v_xor_b32_e64 "):
            continue
        a, b = srcs(out[d])
        between = out[d + 1:k]
        if any(t in srcs(ln) for ln in between + out[k + 1:]):
            continue
        if any(dst(ln) in (a, b) or (dst(ln).startswith("v[") and {a, b} & set(_pair_regs(dst(ln))))
               for ln in between):
            continue
        out[k] = f"v_bitop3_b32 %[{name}], {a}, {b}, %[h0_{'lo' if half == 0 else 'hi'}] bitop3:0x96"
        del out[d]
        counts["v_xor_b32"] -= 2
        counts["v_bitop3_b32"] = counts.get("v_bitop3_b32", 0) + 1
    return out


def uload_layout(base: int, nu: int) -> Dict[int, str]:
    """--uload BASE: SGPR -> the named 32-bit value it holds.  u[i] in s[BASE+2i : BASE+2i+1] (the
    table's byte layout, so three scalar loads fill them); k8, k16 just below BASE and h0_lo, h0_hi
    just above the uniforms (BASE = 36: s34..s71, clear of s32 and of the s72+ that an 8-wave
    kernel reserves)."""
    out: Dict[int, str] = {}
    for i in range(nu):
        out[base + 2 * i] = f"u{i}_lo"
        out[base + 2 * i + 1] = f"u{i}_hi"
    top = base + 2 * nu
    for r, nm in ((base - 2, "k8"), (base - 1, "k16"), (top, "h0_lo"), (top + 1, "h0_hi")):
        out[r] = nm
    return out


def uload_transform(lines: List[str], base: int, nu: int) -> List[str]:
    """The stream reading its uniforms from fixed SGPRs that it loads itself from %[up] (the
    entry's u[] in memory): the compiler then keeps no uniform live across the block, which
    leaves room for 8 waves per SIMD (80 SGPRs).  Prologue: scalar loads, the constants, a wait."""
    assert base % 4 == 0 and nu <= 24
    where = {v: k for k, v in uload_layout(base, nu).items()}
    out = []
    for ln in lines:
        ln = re.sub(r"%\[u(\d+)\]", lambda m: f"s[{base + 2 * int(m.group(1))}:{base + 2 * int(m.group(1)) + 1}]", ln)
        ln = re.sub(r"%\[(u\d+_lo|u\d+_hi|k8|k16|h0_lo|h0_hi)\]", lambda m: f"s{where[m.group(1)]}", ln)
        out.append(ln)
    pro = []
    off = 0
    while off < nu:
        k = min(8, nu - off)
        width = {8: 16, 4: 8, 2: 4, 1: 2}[k] if k in (8, 4, 2, 1) else None
        if width is None:  # split an odd remainder
            k = max(x for x in (8, 4, 2, 1) if x <= k)
            width = 2 * k
        r = base + 2 * off
        pro.append(f"s_load_dwordx{width} s[{r}:{r + width - 1}], %[up], 0x{8 * off:x}")
        off += k
    pro += [f"s_movk_i32 s{where['k8']}, 0x100", f"s_mov_b32 s{where['k16']}, 0x10000",
            f"s_mov_b32 s{where['h0_lo']}, 0x{H0 & M32:08x}", f"s_mov_b32 s{where['h0_hi']}, 0x{H0 >> 32:08x}",
            "s_waitcnt lgkmcnt(0)"]
    return pro + out


def _pair_regs(tok: str) -> List[str]:
    lo, hi = tok[2:-1].split(":")
    return [f"v{r}" for r in range(int(lo), int(hi) + 1)]


# Round 3 (tools/experiments/dual_issue.py): a gfx950 SIMD issues one v_alignbit_b32 per quad-cycle and
# can issue a full-rate instruction of ANOTHER wave in its shadow -- but only when the alignbit's wave
# wins arbitration first (priority, then age); v_lshl_add_u64 hosts no full-rate op (a v_mov_b32 only).
# insert_setprio raises a wave's priority while it runs half-rate instructions, so that a wave in its
# full-rate run fills the shadows of another's alignbits instead of starving it.
SETPRIO_MODES = {"h": {"A": 1, "D": 1, "F": 0}, "a": {"A": 1, "D": 0, "F": 0},
                 "ad": {"A": 2, "D": 1, "F": 0}, "d": {"A": 0, "D": 1, "F": 0}, "da": {"A": 1, "D": 2, "F": 0}}


def insert_setprio(lines: List[str], mode: str) -> List[str]:
    pr = SETPRIO_MODES[mode]
    out, cur = [], 0
    for ln in lines:
        opc = ln.split(" ", 1)[0]
        if opc.startswith("v_"):
            cls = "A" if opc.startswith(("v_alignbit", "v_alignbyte")) else ("D" if opc.startswith(("v_lshl_add_u64", "v_bitop3"))
                                                            else "F")
            want = pr[cls]
            if want != cur:
                out.append(f"s_setprio {want}")
                cur = want
        out.append(ln)
    if cur != 0:
        out.append("s_setprio 0")
    return out


def interpret(lines: List[str], nonce: int, uni_vals: List[int]) -> int:
    regs: Dict[int, int] = {}
    named: Dict[str, int] = {"nonce_lo": nonce & M32, "nonce_hi": nonce >> 32, "k8": 1 << 8, "k16": 1 << 16,
                             "h0_lo": H0 & M32, "h0_hi": H0 >> 32}
    for i, u in enumerate(uni_vals):
        named[f"u{i}_lo"] = u & M32
        named[f"u{i}_hi"] = u >> 32
    # --uload: the uniforms and constants sit in fixed SGPRs (uload_layout), loaded by the block itself
    sregs: Dict[int, int] = {}
    base = next((int(m.group(1)) for ln in lines for m in [re.match(r"s_load_dwordx16 s\[(\d+):", ln)] if m), None)
    if base is not None:
        for k, v in uload_layout(base, len(uni_vals)).items():
            sregs[k] = named[v]

    def rd32(tok: str) -> int:
        tok = tok.strip()
        if tok.startswith("0x"):
            return int(tok, 16)
        if tok.startswith("%["):
            return named[tok[2:-1]]
        if tok.startswith("v") and tok[1:].isdigit():
            return regs[int(tok[1:])]
        if tok.startswith("s") and tok[1:].isdigit():
            return sregs[int(tok[1:])]
        return int(tok)

    def rd64(tok: str) -> int:
        tok = tok.strip()
        if tok == "%[nonce]":
            return nonce
        if tok.startswith("%[u"):
            return uni_vals[int(tok[3:-1])]
        if tok.startswith("s["):
            lo = int(tok[2:-1].split(":")[0])
            return sregs[lo] | (sregs[lo + 1] << 32)
        assert tok.startswith("v["), tok
        lo, hi = tok[2:-1].split(":")
        lo, hi = int(lo), int(hi)
        assert hi == lo + 1 and lo % 2 == 0, tok
        return regs[lo] | (regs[hi] << 32)

    def wr32(tok: str, val: int) -> None:
        tok = tok.strip()
        if tok.startswith("%["):
            named[tok[2:-1]] = val & M32
        else:
            regs[int(tok[1:])] = val & M32

    carry: Dict[str, int] = {}  # "vcc" or "s[k:k+1]" -> the carry bit it holds
    for ln in lines:
        if ln.startswith(".") or ln.startswith("s_"):
            continue  # placement directives / padding / lockstep interval ends / the --uload prologue
        opc, rest = ln.split(" ", 1)
        opc = opc[:-4] if opc.endswith("_e64") else opc
        ops = [t.strip() for t in rest.split(",")]
        if opc == "v_xor_b32":
            wr32(ops[0], rd32(ops[1]) ^ rd32(ops[2]))
        elif opc == "v_bitop3_b32":
            last, mod = ops[3].split(" ", 1)
            assert mod.strip() == "bitop3:0x96", ln  # x ^ y ^ z
            wr32(ops[0], rd32(ops[1]) ^ rd32(ops[2]) ^ rd32(last))
        elif opc == "v_alignbit_b32":
            hi, lo, sh = rd32(ops[1]), rd32(ops[2]), int(ops[3])
            wr32(ops[0], (((hi << 32) | lo) >> sh) & M32)
        elif opc == "v_alignbyte_b32":
            hi, lo, sh = rd32(ops[1]), rd32(ops[2]), int(ops[3])
            wr32(ops[0], (((hi << 32) | lo) >> (8 * (sh & 3))) & M32)
        elif opc == "v_lshrrev_b32":
            wr32(ops[0], rd32(ops[2]) >> int(ops[1]))
        elif opc == "v_mov_b32":
            wr32(ops[0], rd32(ops[1]))
        elif opc == "v_mad_u32_u24":
            wr32(ops[0], (rd32(ops[1]) & 0xffffff) * (rd32(ops[2]) & 0xffffff) + rd32(ops[3]))
        elif opc == "v_add_co_u32":
            assert ops[1] == "vcc" or ops[1].startswith("s[")
            t = rd32(ops[2]) + rd32(ops[3])
            wr32(ops[0], t)
            carry[ops[1]] = t >> 32
        elif opc == "v_addc_co_u32":
            assert ops[1] == "vcc" or ops[1].startswith("s[")
            t = rd32(ops[2]) + rd32(ops[3]) + carry[ops[4]]
            wr32(ops[0], t)
            carry[ops[1]] = t >> 32
        elif opc == "v_lshl_add_u64":
            x = (rd64(ops[1]) << int(ops[2])) & M64
            y = rd64(ops[3])
            s = (x + y) & M64
            lo = int(ops[0][2:-1].split(":")[0])
            regs[lo] = s & M32
            regs[lo + 1] = s >> 32
        else:
            raise ValueError(opc)
    return named["value_lo"] | (named["value_hi"] << 32)


def uniform_values(frontier: List[Node], root_words: List[int]) -> List[int]:
    memo: Dict[int, int] = {}
    return [eval_node(n, 0, root_words, memo) for n in frontier]


# ---------------------------------------------------------------------------------------
def c_expr_program(frontier: List[Node]) -> List[str]:
    """C statements computing every frontier uniform from m[0..3] (host side)."""
    need: Dict[int, Node] = {}
    stack = list(frontier)
    while stack:
        n = stack.pop()
        if n.id in need or n.kind in ("const", "root"):
            continue
        need[n.id] = n
        stack.extend(n.args)

    def ref(n: Node) -> str:
        if n.kind == "const":
            return f"0x{n.val:016x}ull"
        if n.kind == "root":
            return f"m[{n.idx}]"
        return f"t{n.id}"

    out = []
    for nid in sorted(need):
        n = need[nid]
        if n.kind == "add":
            out.append(f"const uint64_t t{nid} = {ref(n.args[0])} + {ref(n.args[1])};")
        elif n.kind == "xor":
            out.append(f"const uint64_t t{nid} = {ref(n.args[0])} ^ {ref(n.args[1])};")
        elif n.kind == "rotr":
            k = n.idx
            out.append(f"const uint64_t t{nid} = ({ref(n.args[0])} >> {k}) | ({ref(n.args[0])} << {64 - k});")
        else:
            raise ValueError(n.kind)
    for i, n in enumerate(frontier):
        out.append(f"u[{i}] = {ref(n)};")
    return out


# Code placement (measured on MI355X, tools/experiments/hash_clock.hip): the same all-8-byte instruction stream
# runs 11 % faster when its instructions sit at byte offsets = 4 (mod 8) than at 0 (mod 8).  The asm
# block therefore opens with ".p2align 3" + one 4-byte s_nop, and every instruction inside it is
# 8 bytes long (VOP3 encodings; VOP2 only with a 32-bit literal), so the parity holds throughout.
PAD = ['.p2align 3', 's_nop 0']


def write_inc(path: str, lines: List[str], frontier: List[Node], host_prog: List[str], vbase: int, vmax: int,
              counts: Dict[str, int], sched: str, est_cycles: float, func: str = "npow_asm_work_value") -> None:
    """The .inc: the host uniform program and the device function.  A second stream of the same
    hash (func != npow_asm_work_value) is device-only: it reads the same uniforms (the frontier does
    not depend on the schedule) and is included after the primary one."""
    nu = len(frontier)
    clobbers = ", ".join(f'"v{r}"' for r in range(vbase, vmax))
    text = "\n".join(lines)
    if "vcc" in text:
        clobbers += ', "vcc"'
    uload = "%[up]" in text
    if uload:  # the fixed SGPRs the block loads its uniforms and constants into
        lo = int(re.search(r"s_load_dwordx16 s\[(\d+):", text).group(1))
        clobbers += "".join(f', "s{k}"' for k in sorted(uload_layout(lo, nu)))
    else:
        for k in sorted({int(m) for m in re.findall(r"s\[(\d+):\d+\]", text)}):
            clobbers += f', "s{k}", "s{k + 1}"'
    ops_in = ['[up] "s"(up)'] if uload else []
    for nm, expr in [("nonce", "nonce"), ("nonce_lo", "(uint32_t)nonce"), ("nonce_hi", "(uint32_t)(nonce >> 32)"),
                     ("k8", "256u"), ("k16", "65536u"),
                     ("h0_lo", f"0x{H0 & M32:08x}u"), ("h0_hi", f"0x{H0 >> 32:08x}u")]:
        if f"%[{nm}]" in text:
            ops_in.append(f'[{nm}] "{"s" if nm.startswith(("k", "h0")) else "v"}"({expr})')
    for i in range(nu):
        if f"%[u{i}]" in text:
            ops_in.append(f'[u{i}] "s"(u[{i}])')
        if f"%[u{i}_lo]" in text:
            ops_in.append(f'[u{i}_lo] "s"((uint32_t)u[{i}])')
        if f"%[u{i}_hi]" in text:
            ops_in.append(f'[u{i}_hi] "s"((uint32_t)(u[{i}] >> 32))')
    uni_ops = ",\n        ".join(ops_in)
    npro = 0
    while uload and not lines[npro].startswith("v_"):
        npro += 1  # the --uload prologue goes before the placement pad: the pad places the VALU stream
    pad = PAD
    if uload and lines[npro - 1] == "s_waitcnt lgkmcnt(0)" and PAD[-1:] == ["s_nop 0"]:
        npro -= 1  # the wait takes the pad's 4-byte s_nop slot: the pad's fill runs while the loads land
        pad = PAD[:-1]
    body = "\n".join(f'      "{ln}\\n"' for ln in lines[:npro] + pad + lines[npro:])
    cnt_txt = ", ".join(f"{k} {v}" for k, v in sorted(counts.items()))
    n_bar = sum(1 for ln in lines if ln.startswith("s_barrier"))
    if func == "npow_asm_work_value":
        prologue = f"""#pragma once
#include <stdint.h>

#define NPOW_ASM_N_UNIFORMS {nu}

// Host: every nonce-independent intermediate the per-lane stream reads.
static inline void npow_asm_uniforms(const uint64_t m[4], uint64_t u[NPOW_ASM_N_UNIFORMS]) {{
{chr(10).join('  ' + s for s in host_prog)}
}}
"""
    else:
        prologue = f"""#pragma once
#include <stdint.h>

static_assert(NPOW_ASM_N_UNIFORMS == {nu}, "include after the primary stream: the same uniforms");
"""
    if uload:
        prologue += f"""
// The block loads the {nu} uniforms itself from `up` (the entry's u[] in memory, 8-byte aligned)
// into fixed SGPRs (tools/gen_hash_asm.py --uload), so none of them is live outside it.
"""
    if n_bar:
        prologue += f"""
// {n_bar} s_barrier: every wave of the workgroup must run this function the same number of
// times, in workgroup-uniform control flow (asm volatile: kept even when a value is unused).
"""
    txt = f"""// GENERATED by tools/gen_hash_asm.py (--sched {sched}) -- do not edit by hand.
//
// gfx950 instruction stream of the Nano work value for one nonce per lane:
//   value = BLAKE2b-64(LE64(nonce) || root)   (nano-work-server.exe @1661643 nano_work)
// Per nonce: {sum(counts.values())} VALU instructions ({cnt_txt});
// VGPR window v{vbase}..v{vmax - 1}; {nu} uniform 64-bit values, {len(ops_in)} asm input operands;
// modelled issue cost {est_cycles:.0f} SIMD cycles per wave (64 nonces).
{prologue}
__device__ __forceinline__ uint64_t {func}(uint64_t nonce, {"const uint64_t* up" if uload else "const uint64_t (&u)[NPOW_ASM_N_UNIFORMS]"}) {{
#if defined(__HIP_DEVICE_COMPILE__)
  uint32_t value_lo, value_hi;
  asm{" volatile" if n_bar else ""}(
{body}
      : [value_lo] "=&v"(value_lo), [value_hi] "=&v"(value_hi)
      : {uni_ops}
      : {clobbers});
  return ((uint64_t)value_hi << 32) | value_lo;
#else
  (void)nonce; (void){"up" if uload else "u"};
  return 0;  // host compilation pass: device code is never executed here
#endif
}}
"""
    with open(path, "w") as f:
        f.write(txt)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--sched", default="seq", choices=["rr", "cp", "seq", "ilp", "lockstep"])
    ap.add_argument("--barrier-nop", action="store_true",
                    help="lockstep: an s_nop 0 after each s_barrier (keeps 8-byte instruction parity)")
    ap.add_argument("--barrier-every", type=int, default=1,
                    help="lockstep: an s_barrier after every N-th interval (0 = none; experiments)")
    ap.add_argument("--func", default="npow_asm_work_value",
                    help="device function name; any other name writes a device-only second stream (write_inc)")
    ap.add_argument("--uload", type=int, default=-1,
                    help="lockstep: the block loads its uniforms into SGPRs from this base on (uload_transform)")
    ap.add_argument("--split", choices=["none", "order", "ad", "fh", "all"], default="none",
                    help="lockstep experiments: adds after alignbits within an interval (SPLIT)")
    ap.add_argument("--shift", action="store_true", help="lockstep: the anti-phase stream (schedule_lockstep)")
    ap.add_argument("--pad-end", action="store_true", help="lockstep: a trailing s_barrier (pairs with --shift)")
    ap.add_argument("--lat", type=float, default=8.0, help="ilp: result latency (SIMD cycles)")
    ap.add_argument("--window", type=int, default=48, help="ilp: scheduling window (instructions)")
    ap.add_argument("--base", type=int, default=16, help="first VGPR of the clobbered window")
    ap.add_argument("--limit", type=int, default=64, help="one past the last VGPR the window may use")
    ap.add_argument("--out", default=os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                                  "nano-dpow_amd", "csrc", "npow_hash_asm.inc"))
    ap.add_argument("--check", type=int, default=64, help="random (root, nonce) pairs to check vs hashlib")
    ap.add_argument("--rotl1", choices=["add", "alignbit", "cc"], default="add",
                    help="rotr63 as v_lshrrev_b32 + v_lshl_add_u64 (add), two v_alignbit_b32, or a "
                         "v_add_co_u32 + 2x v_addc_co_u32 carry chain (cc)")
    ap.add_argument("--add", choices=["u64", "cc", "sgpr"], default="u64",
                    help="64-bit add as one v_lshl_add_u64 (u64) or v_add_co_u32 + v_addc_co_u32 with the "
                         "carry in VCC (cc) or in SGPR pairs taken round-robin (sgpr, --carry-sgprs)")
    ap.add_argument("--carry-sgprs", default="20,22,24,26",
                    help="sgpr: even SGPRs whose pairs carry the adds (round-robin)")
    ap.add_argument("--rotmad", choices=["none", "lo", "hi", "both", "r16", "r24", "r16lo", "r24lo"], default="none",
                    help="rotr16/rotr24 halves as v_lshrrev_b32 + v_mad_u32_u24 instead of v_alignbit_b32")
    ap.add_argument("--enc", choices=["vop3", "vop2"], default="vop3",
                    help="encoding of the simple 32-bit ops (xor, lshrrev)")
    ap.add_argument("--swapmov", action="store_true", help="rotr32 via in-place xors + v_mov_b32 swap")
    ap.add_argument("--fuse-out", choices=["bitop3", "none"], default="bitop3",
                    help="fold the output xors H0 ^ (v0 ^ v8) into v_bitop3_b32 (fuse_output_xor)")
    ap.add_argument("--rotbyte", action="store_true",
                    help="lockstep: rotr24 / rotr16 halves as v_alignbyte_b32 (experiments)")
    ap.add_argument("--alloc", choices=["low", "high", "rr"], default="low",
                    help="lockstep: VGPR allocation order (experiments)")
    ap.add_argument("--run-order", default="id",
                    help="lockstep: op order inside each run -- id, rev, or shufN (seeded); experiments")
    ap.add_argument("--prio", choices=["none", "h", "a", "ad", "d", "da"], default="none",
                    help="s_setprio at instruction-class changes (round 3 experiments, insert_setprio)")
    ap.add_argument("--pad", choices=["odd", "even", "none", "odd64", "even64", "odd128", "even128"], default="odd",
                    help="placement of the stream: 4 (mod 8) [odd], 0 (mod 8) [even], or as it falls; "
                         "odd64 / even64 / odd128 / even128: 4 or 0 bytes past a 64- or 128-byte boundary")
    args = ap.parse_args()
    global ROTL1_VIA_ADD, VOP3_SIMPLE, SWAP_MOV, PAD, ADD_CC, ROTL1_CC
    ADD_CC = args.add == "cc"
    global ADD_SGPR, CARRY_SGPRS
    ADD_SGPR = args.add == "sgpr"
    CARRY_SGPRS = [int(x) for x in args.carry_sgprs.split(",")]
    global ROT_MAD
    ROT_MAD = {"none": lambda n, h: False, "lo": lambda n, h: h == 0, "hi": lambda n, h: h == 1,
               "both": lambda n, h: True, "r16": lambda n, h: n == 16, "r24": lambda n, h: n == 24,
               "r16lo": lambda n, h: n == 16 and h == 0, "r24lo": lambda n, h: n == 24 and h == 0}[args.rotmad]
    SWAP_MOV = args.swapmov
    PAD = {"odd": ['.p2align 3', 's_nop 0'], "even": ['.p2align 3'], "none": [],
           "odd64": ['.p2align 6', 's_nop 0'], "even64": ['.p2align 6'],
           "odd128": ['.p2align 7', 's_nop 0'], "even128": ['.p2align 7']}[args.pad]
    ROTL1_VIA_ADD = args.rotl1 == "add"
    ROTL1_CC = args.rotl1 == "cc"
    VOP3_SIMPLE = args.enc == "vop3"

    dag, out = build_hash_dag()
    ops, frontier, _ = lower(dag, out)
    if args.sched == "ilp":
        ROTL1_VIA_ADD = False
        ins, vrs = lower_ilp(ops, frontier, out)
        order_i = schedule_ilp(ins, args.lat, args.window)
        lines, vmax, counts = allocate_and_emit(order_i, vrs, args.base, args.limit, VOP3_SIMPLE)
    else:
        if args.sched == "lockstep":
            global ZPAIRS, BARRIER_LINES, SPLIT, RUN_ORDER, ALLOC, ROT_BYTE
            ROT_BYTE = args.rotbyte
            SPLIT = args.split
            RUN_ORDER = args.run_order
            ALLOC = args.alloc
            ZPAIRS = 6
            BARRIER_LINES = ["s_barrier", "s_nop 0"] if args.barrier_nop else ["s_barrier"]
            for op in reversed(ops):  # priorities are unused, but keep op.prio defined
                op.prio = 0.0
            order = schedule_lockstep(ops, args.shift, args.pad_end)
            if args.barrier_every != 1:  # experiments: thin out the barriers
                kept, k = [], 0
                for it in order:
                    if it == "BARRIER":
                        k += 1
                        if args.barrier_every == 0 or k % args.barrier_every:
                            continue
                    kept.append(it)
                order = kept
        else:
            order = schedule(ops, args.sched)
        lines, _uni, vmax, counts = emit(order, frontier, out, args.base, args.limit)
    if args.fuse_out == "bitop3":
        lines = fuse_output_xor(lines, counts)
    est = 0.0
    for ln in lines:
        opc = ln.split(" ", 1)[0]
        opc = opc[:-4] if opc.endswith("_e64") else opc
        if opc == "v_xor_b32":
            src0 = ln.split(",")[1].strip()
            est += COST["v_xor_b32_k"] if src0.startswith("0x") else (
                COST["v_xor_b32_s"] if src0.startswith("%[u") else COST["v_xor_b32"])
        elif opc.startswith("s_"):
            continue  # s_barrier / s_nop: not VALU issue
        else:
            est += COST[opc]
    rng = random.Random(2024)
    for _ in range(args.check):
        root = bytes(rng.getrandbits(8) for _ in range(32))
        nonce = rng.getrandbits(64)
        words = [int.from_bytes(root[8 * i:8 * i + 8], "little") for i in range(4)]
        uv = uniform_values(frontier, words)
        got = interpret(lines, nonce, uv)
        want = int.from_bytes(hashlib.blake2b(nonce.to_bytes(8, "little") + root, digest_size=8).digest(), "little")
        if got != want:
            print(f"MISMATCH root={root.hex()} nonce={nonce:016x} got={got:016x} want={want:016x}")
            return 1
    if args.uload >= 0:
        lines = uload_transform(lines, args.uload, len(frontier))
        for _ in range(args.check):  # the transformed stream, interpreted with its SGPR layout
            root = bytes(rng.getrandbits(8) for _ in range(32))
            nonce = rng.getrandbits(64)
            words = [int.from_bytes(root[8 * i:8 * i + 8], "little") for i in range(4)]
            got = interpret(lines, nonce, uniform_values(frontier, words))
            want = int.from_bytes(hashlib.blake2b(nonce.to_bytes(8, "little") + root, digest_size=8).digest(), "little")
            if got != want:
                print(f"MISMATCH (uload) root={root.hex()} nonce={nonce:016x}")
                return 1
    if args.prio != "none":
        lines = insert_setprio(lines, args.prio)
    host_prog = c_expr_program(frontier)
    write_inc(args.out, lines, frontier, host_prog, args.base, vmax, counts, f"{args.sched} --rotl1 {args.rotl1} --add {args.add} --enc {args.enc}"
              + (f" --rotmad {args.rotmad}" if args.rotmad != "none" else "") + (" --swapmov" if args.swapmov else "")
              + (f" --lat {args.lat:g} --window {args.window}" if args.sched == "ilp" else "") + f" --pad {args.pad}"
              + (" --fuse-out none" if args.fuse_out == "none" else "")
              + (f" --func {args.func}" if args.func != "npow_asm_work_value" else "")
              + (f" --uload {args.uload}" if args.uload >= 0 else "")
              + (f" --split {args.split}" if args.split != "none" else "")
              + (f" --run-order {args.run_order}" if args.run_order != "id" else "")
              + (f" --alloc {args.alloc}" if args.alloc != "low" else "")
              + (" --rotbyte" if args.rotbyte else "")
              + (f" --barrier-every {args.barrier_every}" if args.barrier_every != 1 else "")
              + (f" --base {args.base}" if args.base != 16 else "")
              + (f" --limit {args.limit}" if args.limit != 64 else "")
              + (f" --prio {args.prio}" if args.prio != "none" else ""), est, args.func)
    print(f"ops={len(ops)} instrs={len(lines)} {counts} uniforms={len(frontier)} vgpr_window=v{args.base}..v{vmax - 1} "
          f"est_cycles={est:.0f} checked={args.check} -> {os.path.normpath(args.out)}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
