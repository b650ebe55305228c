"""An explicit-state model of the search kernel's entry protocol, checked over every interleaving.

What is modelled (npow_kernel.hip, at the granularity of its shared-memory operations -- each agent-scope atomic or
load completes before the next one of the same wave is issued, ls2_complete, so they are sequentially consistent
among themselves and one step here is one of them):
* two entries E0, E1 of a counted, lingering launch (each in its own slot, one generation), published by the host as
  dynamic entries one after the other (PoolMailbox::ctl, read by lingering workgroups either from the pinned word --
  which also raises the device-memory mirror -- or from the mirror);
* W workgroups, each counted on one of S shards (ls2_shard) of the entry's workgroup counter:
  - ls2_choose (the live entry with the fewest workgroups on the chooser's shard, ties either way; entries seen over
    are marked in the workgroup's s_over mask) and ls2_join (count up, then the dead check; a joiner that finds the
    entry over leaves again through ls2_leave: count down, and the last one out of a dead entry checks every shard
    one after another and publishes);
  - the hash loop: per iteration the top-of-iteration dead load, a hash, optionally a win (ls2_publish_win:
    fetch_max of the dead word, the first raiser publishes the win record), optionally a poll (ls2_poll: the kill
    counter against the launch's relayed key, the kill scan over the launch's entries, the yield word, the entry's
    own kill word, the balancing test), the budget (`late`: the workgroup ends the launch);
  - ls2_leave_wave (the done add, then count down; the last one out of a dead entry reads the shards -- in parallel in
    the kernel, one step each here, in any order with the others' steps -- and publishes the final count);
  - ls2_linger (looks until an entry is new, a yield, or its own budget) and, with RELAY (round 6), its pinned
    looks relaying kills and re-looking at every live entry (ls2_linger_relay);
* the host (npow_pool.cpp): publishes E0 then E1, raises kill words then bumps the kill counter, lets the launch's
  budget pass, and yields only as Worker::step does -- no live slot and no won or killed slot whose final count it
  has not seen.

Checked, over every interleaving (DFS over the explicit states, deduplicated):
* EXACT: on every state, a published final count equals the entry's done total (nothing is added after a publish);
* FIN: from every state where the workgroups all linger or have exited, some still linger (the launch runs on) and an
  entry is won or its kill raised without a published count, a state with that count published is reachable by the
  workgroups' own steps -- the host waits for exactly that before it ends the launch, so otherwise it never would.
The model is test infrastructure (tests/test_pool_protocol_model.py); it stands for the kernel's logic, not its
memory system: stale cache lines, the scalar cache and PCIe ordering are outside it.
"""
from __future__ import annotations

import dataclasses
from typing import Dict, List, Optional, Tuple

HASH_CAP = 1   # hashes counted per segment: 0 or 1 tells a workgroup that hashed from one that did not, which is all the
               # protocol's counts can tell apart (more multiplies the states; the default config was also checked
               # with 2: 2.0 M states, no violation, with and without the relay)


@dataclasses.dataclass(frozen=True)
class Config:
    workgroups: int = 2
    shards: int = 2
    shard_of: Tuple[int, ...] = (0, 1)
    kill: Tuple[bool, ...] = (True, False)   # the host kills entry i (another device won it)
    win: Tuple[bool, ...] = (False, True)    # a workgroup of this device may win entry i
    relay: bool = True                       # round 6: lingering pinned looks relay kills and re-look
    budget: bool = True                      # the launch's time budget may pass (hashing workgroups end)
    linger_timeout: bool = False             # lingering workgroups may reach their own budget and exit
    balance: bool = True                     # polls move a workgroup to a less crowded entry
    entries: int = 2                         # successive dynamic entries (1 or 2; tuples above are indexed by entry)
    # seeded bugs (the checker's own test: each must be caught)
    bug_leave_own_shard: bool = False        # the last leaver checks only its own shard before publishing
    bug_join_no_recheck: bool = False        # a joiner hashes without checking the dead word after its count-up
    bug_kill_no_publish: bool = False        # a relayed kill never publishes (only leavers do)


# shared state ------------------------------------------------------------------------------------------------------
# (dead[2], wgs[2][S], done[2], fin[2] (-1 = none), kill[2], kills, kd, nd, yld, mirror(nd, yld), budget, won[2],
#  killed_host[2] (counter bumped after the kill word))
Shared = tuple
Local = tuple  # (pc, e, local, stop, end, looked, over, tmp, k, attempt, nd_view, sub)


def initial(cfg: Config):
    S, N = cfg.shards, cfg.entries
    shared = ((0,) * N, ((0,) * S,) * N, (0,) * N, (-1,) * N, (0,) * N, 0, 0, 0, 0, (0, 0), 0, (False,) * N, (0,) * N)
    # every workgroup of the launch starts lingering (an empty lingering launch, Worker::launch(true))
    locs = tuple(("LOOK", -1, 0, 0, 0, 0, 0, 0, 0, 0, 0, None) for _ in range(cfg.workgroups))
    return shared, locs


def _set(t, i, v):
    return t[:i] + (v,) + t[i + 1:]


class Model:
    def __init__(self, cfg: Config):
        self.cfg = cfg

    # -- the host -----------------------------------------------------------------------------------------------------
    def host_moves(self, sh, locs) -> List[Tuple[str, Shared]]:
        cfg = self.cfg
        dead, wgs, done, fin, kill, kills, kd, nd, yld, mirror, budget, won, khost = sh
        N_ENT = cfg.entries
        out = []
        if nd < N_ENT and not yld:
            # the next search's entry (dyn_add): the previous one must be decided first (a serial client)
            if nd == 0 or won[nd - 1] or khost[nd - 1]:
                out.append(("pub", _repl(sh, nd=nd + 1)))
        for i in range(N_ENT):
            if i < nd and cfg.kill[i] and not kill[i] and not won[i]:
                # another device won: the watcher raises the kill word (then the counter, below)
                out.append((f"killword{i}", _repl(sh, kill=_set(kill, i, 1))))
            if kill[i] and not khost[i]:
                out.append((f"killcount{i}", _repl(sh, kills=kills + 1, khost=_set(khost, i, 1))))
        if cfg.budget and not budget:
            out.append(("budget", _repl(sh, budget=1)))
        if not yld and nd > 0:
            # Worker::step's end_linger: no live slot (every published entry won or killed) and none draining (each
            # such entry's final count seen)
            over = all(won[i] or khost[i] for i in range(nd))
            drained = all(fin[i] >= 0 for i in range(nd) if won[i] or khost[i])
            if over and drained and nd == N_ENT:
                out.append(("yield", _repl(sh, yld=1)))
        return out

    # -- a workgroup --------------------------------------------------------------------------------------------------
    def wg_moves(self, w: int, sh, loc) -> List[Tuple[str, Shared, Local]]:
        cfg = self.cfg
        dead, wgs, done, fin, kill, kills, kd, nd, yld, mirror, budget, won, khost = sh
        pc, e, local, stop, end, looked, over, tmp, k, attempt, nd_view, sub = loc
        s = cfg.shard_of[w]
        L = lambda **kw: _lrepl(loc, **kw)  # noqa: E731
        out = []
        if pc == "EXIT":
            return out
        if pc == "LOOK":
            # ls2_linger: a pinned read (raises the mirror) or a mirror read
            if cfg.linger_timeout:
                out.append(("linger-timeout", sh, L(pc="EXIT")))
            for pinned in (True, False):
                if pinned:
                    c_nd, c_y = nd, yld
                    sh2 = _repl(sh, mirror=(max(mirror[0], nd), max(mirror[1], yld)))
                else:
                    c_nd, c_y = mirror
                    sh2 = sh
                if c_y:
                    out.append(("look-yield", sh2, L(pc="EXIT")))
                    continue
                if pinned and cfg.relay:
                    # ls2_linger_relay first, then every live entry again
                    out.append(("look-pinned", sh2, L(pc="RELAY", nd_view=c_nd, k=0, looked=0)))
                    continue
                if c_nd > looked:
                    out.append(("look-new", sh2, L(pc="CHOOSE", nd_view=c_nd, attempt=0, looked=looked, e=-1,
                                                   sub="look")))
                elif sh2 != sh:
                    out.append(("look-none", sh2, loc))
            return out
        if pc == "RELAY":
            # ls2_linger_relay: the kill counter against the relayed key, then the scan (one entry per step)
            if k == 0 and sub is None:
                if kills == 0 or kd == kills:
                    return [("relay-skip", sh, L(pc="RELOOK"))]
                return [("relay-start", sh, L(sub=kills))]
            if k >= nd_view:
                return [("relay-end", _repl(sh, kd=sub), L(pc="RELOOK", sub=None, k=0))]
            if (over >> k) & 1 or dead[k] or not kill[k]:
                return [("relay-next", sh, L(k=k + 1))]
            # ls2_kill: fetch_max dead, then the shards one after another (KILLCHK), publish if empty
            return [("relay-kill", _repl(sh, dead=_set(dead, k, 1)),
                     L(pc="KILLCHK", tmp=0, sub=(sub, k, "RELAY")))]
        if pc == "RELOOK":
            if nd_view > 0:
                return [("relook", sh, L(pc="CHOOSE", attempt=0, e=-1, sub="look"))]
            return [("relook-none", sh, L(pc="LOOK"))]
        if pc == "PICK":
            # ls2_pick(!first) in a lingering launch: the entries the device-memory mirror shows, the left one excluded
            return [("pick", sh, L(pc="CHOOSE", nd_view=mirror[0], attempt=0, sub="pick"))]
        if pc == "KILLCHK":
            # ls2_kill's sequential ls2_empty after the fetch_max, for entry ent; then back to the caller
            sub_key, ent, ret = sub
            if cfg.bug_kill_no_publish:
                return [("killchk-skip", sh, _ret(loc, ret, sub_key, ent))]
            if tmp < cfg.shards:
                if wgs[ent][tmp] != 0:
                    return [("killchk-busy", sh, _ret(loc, ret, sub_key, ent))]
                return [("killchk-zero", sh, L(tmp=tmp + 1))]
            return [("kill-publish", _repl(sh, fin=_set(fin, ent, done[ent])), _ret(loc, ret, sub_key, ent))]
        if pc == "CHOOSE":
            fail_looked = nd_view if sub == "look" else 0  # ls2_linger: looked = nd; after ls2_pick: ls2_linger(0)
            if attempt >= 4:
                return [("choose-giveup", sh, L(pc="LOOK", looked=fail_looked, e=-1, sub=None))]
            live = []
            new_over = over
            for i in range(nd_view):
                if (over >> i) & 1 or i == e:
                    continue
                if dead[i]:
                    new_over |= 1 << i
                else:
                    live.append(i)
            if not live:
                return [("choose-none", sh, L(pc="LOOK", looked=fail_looked, over=new_over, e=-1, sub=None))]
            m = min(wgs[i][s] for i in live)
            for i in live:
                if wgs[i][s] == m:  # the pick (lanes' reads); lane 0's join is the next step
                    out.append((f"pick{i}", sh, L(pc="JOINADD", e=i, over=new_over, local=0, stop=0, end=0)))
            return out
        if pc == "JOINADD":
            return [(f"join{e}", _repl(sh, wgs=_inc(wgs, e, s, +1)), L(pc="JOINCHK"))]
        if pc == "JOINCHK":
            if cfg.bug_join_no_recheck:
                return [("join-nocheck", sh, L(pc="HASH"))]
            if dead[e]:
                return [("join-dead", sh, L(pc="JLDEC"))]
            return [("join-live", sh, L(pc="HASH"))]
        if pc == "JLDEC":  # ls2_leave from ls2_join (no done add: it hashed nothing)
            old = wgs[e][s]
            sh2 = _repl(sh, wgs=_inc(wgs, e, s, -1))
            if old == 1:
                return [("jl-dec-last", sh2, L(pc="JLOVER"))]
            return [("jl-dec", sh2, L(pc="CHOOSE", attempt=attempt + 1, e=-1))]
        if pc == "JLOVER":
            if dead[e]:
                return [("jl-over", sh, L(pc="JLEMPTY", tmp=0))]
            return [("jl-live", sh, L(pc="CHOOSE", attempt=attempt + 1, e=-1))]
        if pc == "JLEMPTY":
            if tmp < cfg.shards:
                if wgs[e][tmp] != 0:
                    return [("jl-busy", sh, L(pc="CHOOSE", attempt=attempt + 1, e=-1))]
                return [("jl-zero", sh, L(tmp=tmp + 1))]
            return [("jl-publish", _repl(sh, fin=_set(fin, e, done[e])), L(pc="CHOOSE", attempt=attempt + 1, e=-1))]
        if pc == "HASH":
            # the top of an iteration: the LDS verdict (stop) first
            if stop:
                return [("leave", sh, L(pc="LVADD"))]
            # the dead load, the hash, then the rest of the iteration's decisions
            top_dead = dead[e]
            nl = min(HASH_CAP, local + 1)
            base = L(local=nl, stop=1 if top_dead else 0)
            out.append(("hash", sh, base))
            if cfg.win[e] and not top_dead:
                # ls2_publish_win: fetch_max; the first raiser publishes the win record
                if not dead[e]:
                    out.append(("win", _repl(sh, dead=_set(dead, e, 1), won=_set(won, e, True)), _lrepl(base, stop=2)))
                else:
                    out.append(("win-late", sh, _lrepl(base, stop=2)))
            if not top_dead:
                out.append(("hash-poll", sh, _lrepl(base, pc="POLL", tmp=0, sub=None, k=0)))
            if budget:
                out.append(("hash-late", sh, _lrepl(base, stop=base[3] or 4, end=1)))
            return out
        if pc == "POLL":
            # ls2_poll: the kill counter / key, then the scan of the launch's entries (KILLCHK on a relay)
            if sub is None:
                if kills != 0 and kd != kills:
                    return [("poll-scan", sh, L(sub=("scan", kills), k=0))]
                return [("poll-noscan", sh, L(pc="POLLY"))]
            tag, key = sub[0], sub[1]
            if tag == "scan":
                if k >= nd:
                    return [("poll-scan-end", _repl(sh, kd=key), L(pc="POLLY", sub=None))]
                if (over >> k) & 1 or dead[k] or not kill[k]:
                    return [("poll-scan-next", sh, L(k=k + 1))]
                return [("poll-kill", _repl(sh, dead=_set(dead, k, 1)), L(pc="KILLCHK", tmp=0, sub=(key, k, "SCAN")))]
            return [("poll-?", sh, L(pc="POLLY", sub=None))]
        if pc == "POLLY":
            # the yield word: every live unbounded entry killed (one KILLCHK each), then leave
            if yld:
                for i in range(nd):
                    if not dead[i]:
                        return [("yield-kill", _repl(sh, dead=_set(dead, i, 1)),
                                 L(pc="KILLCHK", tmp=0, sub=(None, i, "YIELD")))]
                return [("yield-leave", sh, L(pc="HASH", stop=3))]
            return [("poll-own", sh, L(pc="POLLOWN"))]
        if pc == "POLLOWN":
            if kill[e]:
                return [("own-kill", _repl(sh, dead=_set(dead, e, 1)), L(pc="KILLCHK", tmp=0, sub=(None, e, "OWN")))]
            if self.cfg.balance:
                # balancing: leave for a live entry with at least two workgroups fewer on this shard
                for i in range(nd):
                    if i != e and not dead[i] and not (over >> i) & 1 and wgs[i][s] + 2 <= wgs[e][s]:
                        return [("balance-leave", sh, L(pc="HASH", stop=3))]
            return [("poll-done", sh, L(pc="HASH"))]
        if pc == "LVADD":  # ls2_leave_wave: the done add, then the count down
            return [("leave-add", _repl(sh, done=_set(done, e, done[e] + local)), L(pc="LVDEC"))]
        if pc == "LVDEC":
            old = wgs[e][s]
            sh2 = _repl(sh, wgs=_inc(wgs, e, s, -1))
            if old == 1:
                return [("leave-dec-last", sh2, L(pc="LVOVER"))]
            return [("leave-dec", sh2, _after_leave(loc))]
        if pc == "LVOVER":
            if dead[e]:
                return [("leave-over", sh, L(pc="LVEMPTY", tmp=0))]
            return [("leave-live", sh, _after_leave(loc))]
        if pc == "LVEMPTY":
            if cfg.bug_leave_own_shard and tmp < cfg.shards and tmp != s:
                return [("leave-skip-shard", sh, L(tmp=tmp + 1))]
            if tmp < cfg.shards:
                if wgs[e][tmp] != 0:
                    return [("leave-busy", sh, _after_leave(loc))]
                return [("leave-zero", sh, L(tmp=tmp + 1))]
            return [("leave-publish", _repl(sh, fin=_set(fin, e, done[e])), _after_leave(loc))]
        raise AssertionError(pc)


def _after_leave(loc):
    pc, e, local, stop, end, looked, over, tmp, k, attempt, nd_view, sub = loc
    if end:  # the budget ended the launch for this workgroup
        return ("EXIT", -1, 0, 0, 0, looked, over, 0, 0, 0, 0, None)
    # ls2_pick(!first): choose over the entries the mirror shows, excluding the one it leaves (PICK)
    return ("PICK", e, 0, 0, 0, 0, over, 0, 0, 0, nd_view, None)


def _ret(loc, ret, key, ent):
    pc, e, local, stop, end, looked, over, tmp, k, attempt, nd_view, sub = loc
    if ret == "RELAY":
        return ("RELAY", e, local, stop, end, looked, over, 0, ent + 1, attempt, nd_view, key)
    if ret == "SCAN":
        return ("POLL", e, local, stop, end, looked, over, 0, ent + 1, attempt, nd_view, ("scan", key))
    if ret == "YIELD":
        return ("POLLY", e, local, stop, end, looked, over, 0, 0, attempt, nd_view, None)
    if ret == "OWN":
        return ("HASH", e, local, 2, end, looked, over, 0, 0, attempt, nd_view, None)
    raise AssertionError(ret)


_FIELDS = ("dead", "wgs", "done", "fin", "kill", "kills", "kd", "nd", "yld", "mirror", "budget", "won", "khost")
_LFIELDS = ("pc", "e", "local", "stop", "end", "looked", "over", "tmp", "k", "attempt", "nd_view", "sub")


def _repl(sh, **kw):
    l = list(sh)
    for name, v in kw.items():
        l[_FIELDS.index(name)] = v
    return tuple(l)


def _lrepl(loc, **kw):
    l = list(loc)
    for name, v in kw.items():
        l[_LFIELDS.index(name)] = v
    return tuple(l)


def _inc(wgs, i, s, d):
    row = list(wgs[i])
    row[s] += d
    assert row[s] >= 0
    return _set(wgs, i, tuple(row))


@dataclasses.dataclass
class Result:
    states: int
    violations: List[Tuple[str, list]]


def check(cfg: Config, max_states: int = 3_000_000, want_trace: bool = True, stop_at_first: bool = False) -> Result:
    """Every interleaving, by DFS over the explicit states (deduplicated), then the properties:
    EXACT on every state; FIN as reachability -- from every state where the workgroups all linger or have exited,
    some linger, and an entry is won or killed without its final count, a state with that count published must be
    reachable by the workgroups' own steps (the host waits for it: without it the launch never ends)."""
    m = Model(cfg)
    start = initial(cfg)
    seen: Dict[tuple, Optional[tuple]] = {start: None}
    stack = [start]
    violations: List[Tuple[str, list]] = []
    kinds = set()
    rev: Dict[tuple, List[tuple]] = {}   # GPU-only edges, reversed
    candidates: List[Tuple[tuple, int]] = []

    def trace(state):
        path = []
        while state is not None:
            prev = seen[state]
            if prev is None:
                break
            path.append(prev[1])
            state = prev[0]
        return path[::-1]

    def report(kind, st):
        if kind not in kinds:
            kinds.add(kind)
            violations.append((kind, trace(st) if want_trace else []))

    N_ENT = cfg.entries
    while stack and not (stop_at_first and violations):
        st = stack.pop()
        sh, locs = st
        dead, wgs, done, fin, kill, kills, kd, nd, yld, mirror, budget, won, khost = sh
        for i in range(N_ENT):
            if fin[i] >= 0 and fin[i] != done[i]:
                report(f"EXACT: entry {i} published {fin[i]}, done {done[i]}", st)
        if all(l[0] in ("LOOK", "EXIT") for l in locs) and any(l[0] == "LOOK" for l in locs):
            for i in range(nd):
                if (won[i] or khost[i]) and fin[i] < 0:
                    candidates.append((st, i))
        succ = []
        for w, loc in enumerate(locs):
            for label, sh2, loc2 in m.wg_moves(w, sh, loc):
                nxt = (sh2, _set(locs, w, loc2))
                if nxt == st:
                    continue
                succ.append((f"w{w}:{label}", nxt))
                rev.setdefault(nxt, []).append(st)
        for label, sh2 in m.host_moves(sh, locs):
            succ.append((f"host:{label}", (sh2, locs)))
        for label, nxt in succ:
            if nxt not in seen:
                seen[nxt] = (st, label)
                stack.append(nxt)
                if len(seen) > max_states:
                    raise RuntimeError(f"state space over {max_states}")
    # FIN: backward reachability over GPU-only edges from the states where entry i's count is published
    for i in range(N_ENT):
        cands = [st for st, j in candidates if j == i]
        if not cands:
            continue
        good = {st for st in seen if st[0][3][i] >= 0}
        frontier = list(good)
        while frontier:
            x = frontier.pop()
            for p in rev.get(x, ()):
                if p not in good:
                    good.add(p)
                    frontier.append(p)
        for st in cands:
            if st not in good:
                won = st[0][11][i]
                report(f"FIN: entry {i} {'won' if won else 'killed'}, a workgroup lingering, no final count ever", st)
                break
    return Result(len(seen), violations)


if __name__ == "__main__":
    import sys
    for relay in (False, True):
        cfg = Config(relay=relay)
        r = check(cfg)
        print(f"relay={relay}: {r.states} states, {len(r.violations)} violation kinds")
        for kind, tr in r.violations:
            print("  ", kind)
            for step in tr:
                print("     ", step)
    sys.exit(0)
