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


@pytest.mark.parametrize("preset,local_rank,want", [(None, 3, "3"), ("0,1,2,3,4,5,6,7", 5, "5"),
                                                    ("4,6", 1, "6"), ("2", 0, "2")])
def test_bench_rank_sees_only_its_gpu(preset, local_rank, want):
    """Under torchrun each bench.py rank must see exactly one GPU: LOCAL_RANK, or the LOCAL_RANK-th
    entry of a device list the launcher already exported (else every rank would search on GPU 0)."""
    import subprocess
    env = {k: v for k, v in os.environ.items() if k != "HIP_VISIBLE_DEVICES"}
    env.update(WORLD_SIZE="8", LOCAL_RANK=str(local_rank), RANK=str(local_rank))
    if preset is not None:
        env["HIP_VISIBLE_DEVICES"] = preset
    out = subprocess.run([sys.executable, "-c", "import os, bench; print(os.environ['HIP_VISIBLE_DEVICES'])"],
                         cwd=ROOT, env=env, capture_output=True, text=True, timeout=120, check=True)
    assert out.stdout.strip() == want


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
