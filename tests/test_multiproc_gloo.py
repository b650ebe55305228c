"""World-size-2 gloo run of bench.py's timed region + reductions (CPU; the GPU search is
replaced by an oracle search).  Checks the contract: value = all ranks' nonces / MAX wall,
ttw gathered from every rank, kernel counters summed; and the per-GPU nonce strides of the
in-process multi-device search are disjoint."""
import os
import socket
import sys

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import ROOT

sys.path.insert(0, ROOT)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import bench
    import oracle
    dist.init_process_group("gloo", rank=rank, world_size=world)

    drawn = []

    def search(i):
        import time
        drawn.append(i)
        t = time.perf_counter()
        scanned, nonce = oracle.search(bench.bench_root(i), 0xffff000000000000, bench.bench_start(i), 1 << 22)
        assert nonce is not None
        return time.perf_counter() - t + (0.01 if rank == 1 else 0.0), scanned

    res = bench.run_timed(search, lambda: (10.0 * (rank + 1), 1000 * (rank + 1), 2), lambda: None,
                          steps=5, warmup=1, rank=rank, world=world, dist=dist)
    line = bench.result_line(world, 5, 1, *res)
    q.put((rank, res, line, drawn[1:]))  # drawn[0] is the rank's warmup search
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_gloo_bench_reduction():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out, timed = {}, []
    for _ in range(2):
        r, res, line, drawn = q.get(timeout=120)
        out[r] = (res, line)
        timed.extend(drawn)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    (n0, w0, ttw0, km0, kn0, l0), line0 = out[0]
    (n1, w1, ttw1, km1, kn1, l1), _ = out[1]
    assert n0 == n1 and w0 == w1          # every rank holds the reduced values
    assert len(ttw0) == 10                # gathered from both ranks
    # the 2 x 5 timed searches came from one node-wide queue: every job root exactly once
    assert sorted(timed) == [1_000_000 + i for i in range(10)]
    assert line0["config"]["searches_total"] == 10
    assert km0 == 30.0 and kn0 == 3000 and l0 == 4
    assert line0["n_gpus"] == 2 and line0["scaling"] == "weak"
    assert line0["value"] == round(n0 / w0 / 1e9, 4)
    assert line0["roofline"]["unit"].startswith("Tops/s")


def test_device_strides_disjoint():
    # npow_search: device k of G starts at start + k * (2^64 / G)  (npow_engine.cpp)
    for G in [1, 2, 3, 4, 8]:
        spacing = ((1 << 64) - 1) // G + 1 if G > 1 else 0
        starts = [(k * spacing) % (1 << 64) for k in range(G)]
        assert len(set(starts)) == G
        if G > 1:
            assert all(b - a >= (1 << 64) // G for a, b in zip(starts, starts[1:]))


@pytest.mark.parametrize("env,local_rank,want", [
    ({}, 3, {"HIP_VISIBLE_DEVICES": "3"}),                                   # nothing exported: device LOCAL_RANK
    ({"HIP_VISIBLE_DEVICES": ""}, 2, {"HIP_VISIBLE_DEVICES": "2"}),          # empty (a GPU-less container): unset
    ({"HIP_VISIBLE_DEVICES": "0,1,2,3,4,5,6,7"}, 5, {"HIP_VISIBLE_DEVICES": "5"}),
    ({"HIP_VISIBLE_DEVICES": "4,6"}, 1, {"HIP_VISIBLE_DEVICES": "6"}),
    ({"HIP_VISIBLE_DEVICES": "2"}, 0, None),                                 # already one device: kept
    ({"CUDA_VISIBLE_DEVICES": "3"}, 3, None),                                # a launcher narrowed CUDA_...
    ({"CUDA_VISIBLE_DEVICES": "4,5"}, 1, {"HIP_VISIBLE_DEVICES": "5"}),
    ({"ROCR_VISIBLE_DEVICES": "6"}, 6, None),                                # ... or ROCR_: HIP sees one
    ({"ROCR_VISIBLE_DEVICES": "1,3,5,7"}, 2, {"HIP_VISIBLE_DEVICES": "2"}),  # index into ROCR's list
    ({"ROCR_VISIBLE_DEVICES": "1,3", "HIP_VISIBLE_DEVICES": "0,1"}, 1, {"HIP_VISIBLE_DEVICES": "1"}),
])
def test_rank_visibility_presets(env, local_rank, want):
    """Under torchrun each bench.py rank must see exactly one GPU: its own if a launcher already
    narrowed HIP_/CUDA_/ROCR_VISIBLE_DEVICES to one, else the LOCAL_RANK-th visible device."""
    import bench
    assert bench.rank_visibility(env, local_rank) == want


@pytest.mark.parametrize("env,local_rank", [({"HIP_VISIBLE_DEVICES": "0,1"}, 2), ({"ROCR_VISIBLE_DEVICES": "4,5"}, 3)])
def test_rank_visibility_too_few_devices_fails(env, local_rank):
    import bench
    with pytest.raises(SystemExit):
        bench.rank_visibility(env, local_rank)


def test_bench_rank_environment_is_applied_at_import():
    """The rank's visibility is set when bench.py is imported, before anything can open the GPU."""
    import subprocess
    env = {k: v for k, v in os.environ.items() if not k.endswith("_VISIBLE_DEVICES")}
    env.update(WORLD_SIZE="8", LOCAL_RANK="5", RANK="5", HIP_VISIBLE_DEVICES="0,1,2,3,4,5,6,7")
    out = subprocess.run([sys.executable, "-c", "import os, bench; print(os.environ['HIP_VISIBLE_DEVICES'])"],
                         cwd=ROOT, env=env, capture_output=True, text=True, timeout=120, check=True)
    assert out.stdout.strip() == "5"


def test_bench_gpus_must_match_world_size():
    """--gpus N under torchrun must equal WORLD_SIZE: a mismatch exits non-zero before any GPU work."""
    import subprocess
    env = {k: v for k, v in os.environ.items() if not k.endswith("_VISIBLE_DEVICES")}
    env.update(WORLD_SIZE="2", LOCAL_RANK="0", RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT="1")
    p = subprocess.run([sys.executable, "bench.py", "--gpus", "4", "--no-cpu-baseline"], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=120)
    assert p.returncode != 0 and "WORLD_SIZE=2" in p.stderr


def _node_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import bench
    from fake_engine import OracleEngine
    dist.init_process_group("gloo", rank=rank, world_size=world)
    # rank 1 is slow (sleeps between chunks), so rank 0 wins most roots and must cancel rank 1
    eng = OracleEngine(chunk=1 << 10, delay=0.0 if rank == 0 else 0.002)
    out = bench.node_time_to_work(eng, 0, rank, world, dist, 12, thr=0xfff0000000000000)
    q.put((rank, out, [(c[2] % (1 << 64)) for c in eng.calls]))
    dist.barrier()
    dist.destroy_process_group()


def test_node_time_to_work_cross_rank_first_win():
    """bench.node_time_to_work: every root searched by both ranks on disjoint strides, the first win
    cancelling the other rank's search through the shared-memory word."""
    import glob
    import tempfile
    pattern = os.path.join(tempfile.gettempdir(), "nanopow_bench_cancel_*")
    before = set(glob.glob(pattern))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_node_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = {}
    for _ in range(2):
        r, out, starts = q.get(timeout=180)
        got[r] = (out, starts)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    out = got[0][0]
    assert got[1][0] is None and out["n"] == 12 and out["failed"] == 0 and out["shared_cancel"]
    assert out["p50"] > 0 and out["p99"] >= out["p50"]
    assert out["node_gnps"] > 0 and out["nonces_per_search"] > 0
    assert out["rank_searches_cancelled"] >= 6  # the slow rank is cancelled by the winner's word
    # disjoint strides: rank 1 starts half the nonce space away from rank 0, root by root
    for s0, s1 in zip(got[0][1], got[1][1]):
        assert (s1 - s0) % (1 << 64) == 1 << 63
    assert set(glob.glob(pattern)) == before  # the shared file is unlinked at the end


def test_inprocess_multi_gpu_path_with_oracle_engine():
    """bench.py --gpus N without torchrun: N searches in flight over the pool's N-device mask, each
    split into N disjoint strides (here the oracle stand-in emulates the split), every one returning a
    valid winner; value = all nonces / wall, the timed searches' overshoot summarised, then one root
    at a time over all N (node_ttw_ms)."""
    import bench
    import oracle
    from fake_engine import OracleEngine
    eng = OracleEngine(chunk=1 << 10, n_devices=2)
    thr = 0xfff0000000000000
    nonces, wall, ttw, recs, kern_ms, kern_nonces, launches, ks = bench.run_timed_inprocess(eng, 2, 4, 1, thr=thr)
    assert len(ttw) == 8 and nonces == sum(r[1] for r in recs) and nonces == kern_nonces > 0
    line = bench.result_line(2, 4, 1, nonces, wall, ttw, kern_ms, kern_nonces, launches, parallelism="in-process x2")
    assert line["n_gpus"] == 2 and line["config"]["searches_total"] == 8
    assert line["value"] == round(nonces / wall / 1e9, 4)
    node = bench.inprocess_node_ttw(eng, 2, 6, thr=thr)
    assert node["n"] == 6 and node["p99"] >= node["p50"] > 0
    assert "stop_after_decide_us" in node and "overshoot_nonces" in node
    # the emulated split searched both strides of every root
    starts = {}
    for root, t, start in eng.calls:
        starts.setdefault(root, set()).add(start)
    assert all(len(v) == 2 for v in starts.values())
    for root, v in starts.items():
        a, b = sorted(v)
        assert (b - a) % (1 << 64) == 1 << 63 or (a - b) % (1 << 64) == 1 << 63
    assert oracle.work_value(root, 0) >= 0  # the checker is importable here


def test_regime_harness_with_oracle_engine():
    """bench.py --workload regime on the oracle stand-in over 2 emulated devices: one root at a time,
    the next submitted at the previous result, tickets collected by the reaper; the record's rates, expectation and
    fixed-cost decomposition are filled in, and the device check passes on equal, fully counted devices."""
    import bench
    from fake_engine import OracleEngine
    eng = OracleEngine(chunk=1 << 10, n_devices=2)
    rec = bench.node_regime(eng, 2, 12, thr=0xfff0000000000000)
    assert rec["devices"] == 2 and rec["searches"] == 12 and rec["threshold"] == "fff0000000000000"
    assert rec["c_abi_ttw_ms"]["p99"] >= rec["c_abi_ttw_ms"]["p50"] > 0
    assert rec["kernel_gnps"] > 0 and rec["node_gnps"] > 0 and rec["expected_p50_ms"] > 0
    f = rec["fixed_cost_us"]
    assert abs(f["per_search_wall_us"] - f["hashing_at_kernel_rate_us"] - f["fixed_us"]) < 0.2
    d = rec["decomposition_us"]
    for k in ("gpu_idle_between_launches", "decided_to_result_in_client", "client_turnaround_to_next_submit",
              "losers_stop_after_decide"):
        assert k in d
    chk = bench.device_check([4.3, 4.31, 4.29], 1000, 1000)
    assert chk["ok"] and chk["slow_devices"] == []
    bad = bench.device_check([4.3, 4.31, 3.5], 1000, 1000)
    assert not bad["ok"] and bad["slow_devices"] == [2]
    assert not bench.device_check([4.3, 4.3], 999, 1000)["ok"]  # counters that do not sum
    # per MHz when the clocks are known: a GPU at a lower power-capped clock is no fault, a slow one at its clock is
    assert bench.device_check([35.0, 32.4], 10, 10, [2340.0, 2170.0])["ok"]
    assert bench.device_check([35.0, 35.0, 31.0], 10, 10, [2340.0] * 3)["slow_devices"] == [2]
