"""Child process of tests/test_gpu_multidevice.py: first-found cancellation across devices
(north_star; the work_cancel -> {"error": "Cancelled"} semantics of nano-work-server.exe @1673856,
client/work_handler.py:61-80).  Run with NANOPOW_VIRTUAL_DEVICES=G: searches split over all G
devices (disjoint strides); for each, npow_wait_info reports when the host accepted the winner and
how long the other devices kept hashing after that (host-observed upper bound) with the nonces that
span is worth at each device's kernel rate, and the nonces the losing devices' waves hashed after they
knew the job was over, counted in the kernel (late_nonces_losers).  Asserts a valid winner every time and a bound on the
overshoot; prints one JSON line with the distributions."""
import json
import os
import random
import statistics
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(ROOT, "nano-dpow_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import oracle  # noqa: E402  (the checker)
from nanopow import _lib  # noqa: E402

THRESHOLDS = {"send": 0xfffffff800000000, "receive": 0xfffffe0000000000}


def pct(xs, p):
    xs = sorted(xs)
    return xs[min(len(xs) - 1, max(0, int(round(p / 100.0 * (len(xs) - 1)))))]


def main(n_search, which, mask=0):
    """mask != 0: split every search over those devices only (the others idle): e.g. 4 of 8 CU partitions, to tell
    the engine's stop path from the hardware queues' scheduling of 5+ concurrently busy CU-masked queues."""
    eng = _lib.Engine()
    G = eng.n_devices if not mask else bin(mask).count("1")
    thr = THRESHOLDS[which]
    rng = random.Random(11)
    spans, over, done, ttw, winners, late_l, late_w, res_ms = [], [], [], [], [], [], [], []
    for i in range(n_search):
        root = bytes(rng.getrandbits(8) for _ in range(32))
        t0 = time.perf_counter()
        t = eng.submit(root, thr, start=rng.getrandbits(64), device_mask=mask)
        r = t.wait_result(120)  # the outcome at the decision (what a client is answered with)
        res_ms.append((time.perf_counter() - t0) * 1e3)
        info = t.wait_info(120)
        assert r.status == info.status and r.nonce == info.nonce
        assert info is not None and info.status == _lib.NPOW_OK, info
        assert oracle.work_value_hashlib(root, info.nonce) == info.value >= thr
        assert info.n_devices == G and 0 <= info.winner_device < eng.n_devices
        assert not mask or (mask >> info.winner_device) & 1
        spans.append(info.stop_after_decide_us)
        over.append(info.overshoot_nonces)
        late_l.append(info.late_nonces_losers)
        late_w.append(info.late_nonces_winner)
        done.append(info.nonces_done)
        ttw.append(info.finish_us)
        winners.append(info.winner_device)
    st = [eng.stats(d) for d in range(eng.n_devices) if not mask or (mask >> d) & 1]
    kills = sum(x.kills_relayed for x in st)
    # the losers' late hashes are deterministic: in each losing device's one-entry launch every workgroup but the
    # one whose poll read the kill word sees the relayed dead word before a hash and leaves after it -- one hash of
    # 512 lanes (npow_kernel.hip pool_body_ls2, kind 1) -- while the relaying workgroup leaves at once (kind 2)
    grid = st[0].grid
    late_expected = (G - 1) * (grid - 1) * 512 if all(x.grid == grid for x in st) else None
    res = {"ok": True, "devices": G, "threshold": which, "searches": n_search,
           "partitions": [[x.hip_device, x.cu_first, x.cus] for x in st],
           "stop_after_decide_us": {"p50": round(pct(spans, 50), 1), "p99": round(pct(spans, 99), 1),
                                    "max": round(max(spans), 1)},
           "overshoot_nonces": {"p50": pct(over, 50), "p99": pct(over, 99),
                                "mean_over_nonces_done": round(sum(over) / max(1, sum(done)), 5)},
           # counted in the kernels: the losing devices' hashes after their waves knew the job was over
           "late_nonces_losers": {"p50": pct(late_l, 50), "p99": pct(late_l, 99),
                                  "mean_over_nonces_done": round(sum(late_l) / max(1, sum(done)), 5)},
           "late_nonces_winner": {"p50": pct(late_w, 50), "p99": pct(late_w, 99)},
           "late_expected": late_expected, "grid_per_device": grid,
           "late_equal_share": round(sum(1 for x in late_l if x == late_expected) / len(late_l), 4),
           "late_max": max(late_l),
           "affinity": [sum(x.affinity_checks for x in st), sum(x.affinity_failures for x in st)],
           # one iteration of each device's grid (one 64-nonce hash per wave, 512 nonces per workgroup) at its kernel
           # rate over the time it hashed (kernel_ms less its lingering launches' idle waits, npow_device_stats ABI 6)
           "iteration_us": [round(x.grid * 512 / (x.nonces / max(1e-9, x.kernel_ms - x.linger_ms) / 1e3), 2)
                            for x in st],
           "stale_drains": sum(x.stale_drains for x in st),
           "linger_relays": sum(x.linger_relays for x in st),
           "stale_late": sum(x.stale_late for x in st), "stale_missing": sum(x.stale_missing for x in st),
           "stale_gpu_delay_us": round(max(x.stale_gpu_delay_us for x in st), 1),
           "linger": os.environ.get("NANOPOW_LINGER", "default"),
           "finish_ms_p50": round(pct(ttw, 50) / 1e3, 3),
           "result_ms_p50": round(pct(res_ms, 50), 3),
           "distinct_winners": len(set(winners)), "kills_relayed": kills,
           "mean_nonces_done": round(statistics.mean(done))}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main(int(sys.argv[1]), sys.argv[2], int(sys.argv[3], 0) if len(sys.argv) > 3 else 0)
