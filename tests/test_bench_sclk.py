"""bench.py's shader-clock sampler (host logic; CPU).  On the GPU box it reads the GPU's own
pp_dpm_sclk; here a file of the same format stands in for it."""
import os
import sys
import time

from conftest import ROOT

sys.path.insert(0, ROOT)
import bench  # noqa: E402


def test_sampler_reads_the_current_level(tmp_path):
    f = tmp_path / "pp_dpm_sclk"
    f.write_text("0: 500Mhz\n1: 2387Mhz *\n2: 2400Mhz\n")
    s = bench.SclkSampler(0, period=0.005)
    s.path, s.bus = str(f), "0000:a7:00.0"
    with s:
        time.sleep(0.05)
        f.write_text("S: 95Mhz *\n0: 500Mhz\n1: 2400Mhz\n")
        time.sleep(0.05)
    out = s.summary()
    assert out["max"] == 2387 and out["min"] == 95 and out["samples"] >= 4
    assert "0000:a7:00.0" in out["source"]


def test_sampler_without_sysfs_reports_nothing():
    s = bench.SclkSampler(0)
    s.path = None
    with s:
        pass
    assert s.summary() is None


def test_cpu_baseline_is_hashlib_on_every_granted_core():
    """cpu_baseline: hashlib (the reference CPU path) in one process per granted core over disjoint
    ranges; its hit set equals the C oracle's over the same range."""
    out = bench.cpu_baseline(seconds=0.3)
    assert out["kind"] == "reference" and out["cores"] == bench.granted_cores()
    assert out["value"] > 0 and out["port_gnps"] > out["value"] and out["hits_equal_port"]
    assert "hashlib.blake2b(digest_size=8)" in out["sample"]
