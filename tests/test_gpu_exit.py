"""Process exit with launches in flight.

Round 5 found processes running lingering launches dying with SIGSEGV in their exit handlers under rocprofv3
(profiles/r05aq_hip_api_trace_overshoot_g4.txt; the bench's regime child, tools/prof_r04.sh): at exit the pool
workers left at once, and a lingering launch (or a search launch) was still running while the HIP runtime and the
profiler's tool library tore down.  Since round 6 the exit hook drains like npow_shutdown -- every job cancelled, its
kill word raised, lingering launches given their yield, every launch retired -- before the runtime's own exit handlers
run, and then frees every device's streams, events and memory as npow_shutdown does (npow_pool.cpp pool_exit,
npow_engine.cpp's exit hook): round 6's first run showed the crash with the drain alone -- after rocprofv3's tool
finalisation, in a static destructor (profiles/r06a_exit_sigsegv.txt), i.e. in the runtime's teardown of the process's
CU-masked streams.  Checked here: the overshoot worker over 4 CU partitions with lingering launches forced on and off,
and the bench's 8-partition regime child (lingering on by default there), exit with rc 0 on their own and under
`rocprofv3 --kernel-trace --stats`, each ending while the engine still has launches running (the process exits right
after its last search, without npow_shutdown).
Run on an MI355X: ``pytest -m gpu``.
"""
import os
import shutil
import subprocess
import sys
import tempfile

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu

ROCPROF = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"


def _run(cmd, env_extra, profiled, timeout=150):
    env = dict(os.environ, TMPDIR="/tmp", **env_extra)
    out_dir = tempfile.mkdtemp(prefix="npow_exit_", dir="/tmp")
    try:
        if profiled:
            if not os.path.exists(ROCPROF):
                pytest.skip("rocprofv3 not found")
            cmd = [ROCPROF, "--kernel-trace", "--stats", "--output-format", "csv", "-d", out_dir, "-o", "run", "--", *cmd]
        try:
            p = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=timeout)
        except subprocess.TimeoutExpired as e:  # (a hang at exit: report what it printed)
            err = e.stderr.decode(errors="replace") if isinstance(e.stderr, bytes) else (e.stderr or "")
            out = e.stdout.decode(errors="replace") if isinstance(e.stdout, bytes) else (e.stdout or "")
            pytest.fail(f"timed out after {timeout} s; stdout {out[-600:]!r}; stderr {err[-4000:]!r}")
        traced = []
        for base, _dirs, files in os.walk(out_dir):
            traced += [f for f in files if f.endswith(".csv")]
    finally:
        shutil.rmtree(out_dir, ignore_errors=True)
    return p, traced


OVERSHOOT = [sys.executable, os.path.join("tests", "overshoot_worker.py"), "100", "receive"]
PARTITIONS = {"linger4": {"NANOPOW_LINGER": "1", "NANOPOW_VIRTUAL_DEVICES": "4"},   # lingering launches at exit
              "cu4": {"NANOPOW_LINGER": "0", "NANOPOW_VIRTUAL_DEVICES": "4"}}      # CU-masked streams, no lingering
REGIME = [sys.executable, "bench.py", "--workload", "regime", "--gpus", "8", "--steps", "200", "--http-requests", "20"]
REGIME_ENV = {"NANOPOW_VIRTUAL_DEVICES": "8"}


@pytest.mark.parametrize("profiled", [False, True], ids=["plain", "rocprofv3"])
@pytest.mark.parametrize("parts", sorted(PARTITIONS))
def test_partitioned_overshoot_worker_exits_cleanly(parts, profiled):
    p, traced = _run(OVERSHOOT, PARTITIONS[parts], profiled)
    assert p.returncode == 0, (p.returncode, p.stdout[-1500:], p.stderr[-3000:])
    assert '"ok": true' in p.stdout
    if profiled:
        assert traced, "rocprofv3 wrote no trace"


@pytest.mark.parametrize("profiled", [False, True], ids=["plain", "rocprofv3"])
def test_regime_child_exits_cleanly(profiled):
    p, traced = _run(REGIME, REGIME_ENV, profiled)
    assert p.returncode == 0, (p.returncode, p.stdout[-1500:], p.stderr[-3000:])
    assert "node_ttw_8x_regime" in p.stdout
    import json
    rec = json.loads(p.stdout.strip().splitlines()[-1])["node_ttw_8x_regime"]
    assert rec["stale_final_counts"]["missing"] == 0, rec["stale_final_counts"]  # no final count lost
    if profiled:
        assert traced, "rocprofv3 wrote no trace"


def test_work_server_stops_on_sigterm_with_searches_running():
    """`python -m nanopow` under systemd is stopped with SIGTERM: the server turns it into an orderly stop (the pending
    work_generate requests answered {"error": "Cancelled"}, the listener closed) and a normal exit, so the library's exit
    hook drains and frees the GPU -- rc 0, not death by signal with launches in flight."""
    import json
    import signal
    import socket
    import threading
    import time
    import urllib.request
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ, PYTHONPATH=os.path.join(ROOT, "nano-dpow_amd"))
    p = subprocess.Popen([sys.executable, "-m", "nanopow", "-l", f"127.0.0.1:{port}"], cwd=ROOT, env=env,
                         stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    try:
        deadline = time.time() + 90
        ready = False
        while time.time() < deadline and not ready:
            line = p.stderr.readline()
            if not line:
                break
            ready = "Ready to receive requests" in line
        assert ready, "the work server did not come up"
        replies = []

        def generate(i):
            body = json.dumps({"action": "work_generate", "hash": f"{i + 7:064x}", "difficulty": "ffffffffffffffff"})
            req = urllib.request.Request(f"http://127.0.0.1:{port}", data=body.encode(), method="POST",
                                         headers={"Content-Type": "application/json"})
            try:
                with urllib.request.urlopen(req, timeout=30) as r:
                    replies.append(json.loads(r.read()))
            except Exception as e:  # (a reply cut off by the exit would land here; recorded)
                replies.append({"exception": repr(e)})

        ths = [threading.Thread(target=generate, args=(i,), daemon=True) for i in range(2)]
        for t in ths:
            t.start()
        time.sleep(0.5)  # both searches running (endless at this threshold)
        p.send_signal(signal.SIGTERM)
        rc = p.wait(30)
        for t in ths:
            t.join(10)
    finally:
        if p.poll() is None:
            p.kill()
            p.wait(10)
    assert rc == 0, (rc, p.stderr.read()[-3000:])
    assert replies and all(r == {"error": "Cancelled"} for r in replies), replies
