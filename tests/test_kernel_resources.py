"""The shipped gfx950 kernels fit the shape they are launched with (CPU test, no GPU).

The search, sweep and values kernels run 8 waves per SIMD (four 512-lane workgroups per CU), which
needs <= 64 VGPRs and no AGPRs per wave (512 per SIMD lane / 8), and their loops must not touch
scratch: a spill there is a slower kernel that still passes every parity test.  This reads the AMDHSA
metadata of the gfx950 code object inside the built libnanopow.so (.hip_fatbin section, unbundled with
the ROCm LLVM tools) and checks every kernel's .vgpr_count, .agpr_count and
.private_segment_fixed_size.
"""
import os
import re
import subprocess

import pytest

from conftest import ROOT

LLVM = "/opt/rocm/lib/llvm/bin"
LIB = os.path.join(ROOT, "nano-dpow_amd", "nanopow", "libnanopow.so")
EIGHT_WAVES = ("npow_pool_kernel_ls2", "npow_sweep_kernel_ls2", "npow_values_kernel_ls2")


def kernel_metadata(tmp_path):
    fat, co = tmp_path / "fat.bin", tmp_path / "k.co"
    subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", LIB, str(tmp_path / "lib.tmp")],
                   check=True, capture_output=True)
    subprocess.run([f"{LLVM}/clang-offload-bundler", "--type=o", "--targets=hipv4-amdgcn-amd-amdhsa--gfx950",
                    f"--input={fat}", f"--output={co}", "--unbundle"], check=True, capture_output=True)
    notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", str(co)], check=True, capture_output=True,
                           text=True).stdout
    kernels = {}
    for block in notes.split("  - .agpr_count:")[1:]:
        fields = dict(re.findall(r"\.(\w+):\s+(\S+)", ".agpr_count:" + block))
        if "name" in fields and "vgpr_count" in fields:
            kernels[fields["name"]] = {k: int(fields[k]) for k in ("agpr_count", "vgpr_count", "sgpr_count",
                                                                   "private_segment_fixed_size")}
    return kernels


@pytest.mark.skipif(not (os.path.exists(LIB) and os.path.exists(f"{LLVM}/clang-offload-bundler")),
                    reason="libnanopow.so not built or no ROCm LLVM tools")
def test_shipped_kernels_fit_eight_waves_per_simd_without_scratch(tmp_path):
    kernels = kernel_metadata(tmp_path)
    shipped = {n: m for n, m in kernels.items() if any(k in n for k in EIGHT_WAVES)}
    # search (bounded / unbounded, table in kernel arguments or in memory), sweep, values
    assert len(shipped) == 6, sorted(kernels)
    for name, m in shipped.items():
        assert m["vgpr_count"] <= 64 and m["agpr_count"] == 0, (name, m)
        assert m["private_segment_fixed_size"] == 0, (name, m)  # no scratch
    for name, m in kernels.items():
        assert m["private_segment_fixed_size"] == 0, (name, m)
