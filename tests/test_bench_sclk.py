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
