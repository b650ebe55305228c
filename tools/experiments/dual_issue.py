#!/usr/bin/env python3
"""Which VALU instruction classes dual-issue on a gfx950 SIMD (round 3).

SQ_ACTIVE_INST_VALU2 counts "quad-cycles two VALU instructions are issued" per SIMD: in the search
kernel 44 % of quad-cycles carry two (profiles/r03_pmc_dual_issue.json).  This probe runs two
1,024-lane workgroups per CU (8 waves per SIMD, as the search kernel) where waves 0-7 of every
workgroup repeat one instruction class and waves 8-15 another, all instructions independent, until
a common wall-clock budget; one kernel per (class A, class B) pair, so rocprofv3 --pmc attributes
the counters per pair.  Each kernel also reports, from the waves' own counts, instructions per
SIMD-cycle for each half.

  python3 tools/experiments/dual_issue.py build      -> build/dual_issue (hipcc, gfx950)
  build/dual_issue [budget_us]                       -> one JSON line per pair (GPU box)
DUAL_PAIRS=DA,DP,... picks the pairs, DUAL_TAG=name suffixes the binary (round 3: the reverse orders).
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
TAG = os.environ.get("DUAL_SPLIT", "half") + ("_" + os.environ["DUAL_TAG"] if os.environ.get("DUAL_TAG") else "")
SRC = os.path.join(ROOT, "build", "dual_issue_%s.hip" % TAG)
BIN = os.path.join(ROOT, "build", "dual_issue_%s" % TAG)

CLASSES = {
    "X": lambda d, a, b: f"v_xor_b32 v{d}, v{a}, v{b}",
    "E": lambda d, a, b: f"v_xor_b32_e64 v{d}, v{a}, v{b}",
    "A": lambda d, a, b: f"v_alignbit_b32 v{d}, v{a}, v{b}, 24",
    "Y": lambda d, a, b: f"v_alignbyte_b32 v{d}, v{a}, v{b}, 3",
    "R": lambda d, a, b: f"v_perm_b32 v{d}, v{a}, v{b}, s8",
    "D": lambda d, a, b: f"v_lshl_add_u64 v[{d & ~1}:{(d & ~1) + 1}], v[{a & ~1}:{(a & ~1) + 1}], 0, v[{b & ~1}:{(b & ~1) + 1}]",
    "L": lambda d, a, b: f"v_lshrrev_b32 v{d}, 31, v{a}",
    "M": lambda d, a, b: f"v_mov_b32 v{d}, v{a}",
    "P": lambda d, a, b: f"v_add_u32 v{d}, v{a}, v{b}",
    "B": lambda d, a, b: f"v_bitop3_b32 v{d}, v{a}, v{b}, v{(b + 2) % 24 + 24} bitop3:0x96",
    "N": None,  # no VALU: the other half alone
}
PAIRS = os.environ.get("DUAL_PAIRS", "").split(",") if os.environ.get("DUAL_PAIRS") else ["XX", "AA", "DD", "LL", "XA", "XD", "AD", "LA", "LD", "MA", "MD", "PA", "PD", "EA", "ED", "BA", "BD",
         "XN", "AN", "DN", "AX", "DX"]
# SPLIT: which waves run class A.  "half": waves 0-7 of a workgroup (older) vs 8-15; "alt": waves whose
# index has bit 2 clear vs set -- every SIMD (wave w -> SIMD w % 4) then holds both classes in
# alternating age order.
SPLIT = os.environ.get("DUAL_SPLIT", "half")
N_INST = 64


def body(c):
    if CLASSES[c] is None:
        return '"s_nop 0\\n"'
    lines = []
    for i in range(N_INST):
        d = 8 + (2 * i) % 16 if c == "D" else 8 + i % 16
        a, b = 24 + (2 * i) % 24, 24 + (2 * i + 6) % 24
        lines.append('"' + CLASSES[c](d, a, b) + '\\n"')
    return "\n          ".join(lines)


def gen():
    clob = ", ".join(f'"v{r}"' for r in range(8, 48))
    ks = []
    for p in PAIRS:
        ks.append(f"""
__global__ __launch_bounds__(1024, 8) void k_{p}(uint64_t budget, unsigned long long* out) {{
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  const uint64_t c0 = __builtin_amdgcn_s_memtime();
  const unsigned wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  unsigned long long it = 0;
  if ({'wave < 8' if SPLIT == 'half' else '(wave & 4) == 0'}) {{
    while (__builtin_amdgcn_s_memrealtime() - t0 < budget) {{
      asm volatile({body(p[0])} ::: {clob});
      ++it;
    }}
  }} else {{
    while (__builtin_amdgcn_s_memrealtime() - t0 < budget) {{
      asm volatile({body(p[1])} ::: {clob});
      ++it;
    }}
  }}
  const uint64_t c1 = __builtin_amdgcn_s_memtime();
  if ((threadIdx.x & 63) == 0) {{
    atomicAdd(&out[({'wave < 8' if SPLIT == 'half' else '(wave & 4) == 0'}) ? 0 : 1], it);
    if (blockIdx.x == 0 && wave == 0) {{ out[2] = c1 - c0; out[3] = __builtin_amdgcn_s_memrealtime() - t0; }}
  }}
}}""")
    runs = "\n".join(f'  run("{p}", k_{p}, budget, cus);' for p in PAIRS)
    return f"""#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <stdlib.h>
{''.join(ks)}
template <class K>
static void run(const char* name, K kern, uint64_t budget, int cus) {{
  unsigned long long* d; hipMalloc(&d, 4 * 8); hipMemset(d, 0, 4 * 8);
  hipLaunchKernelGGL(kern, dim3(cus * 2), dim3(1024), 0, 0, budget, d);
  unsigned long long h[4]; hipMemcpy(h, d, 32, hipMemcpyDeviceToHost); hipFree(d);
  const double cyc = (double)h[2], simds = cus * 4.0;
  printf("{{\\"pair\\": \\"%s\\", \\"ipc_a\\": %.4f, \\"ipc_b\\": %.4f, \\"ipc\\": %.4f, \\"cycles\\": %.0f, \\"mhz\\": %.1f}}\\n",
         name, h[0] * {N_INST}.0 / simds / cyc, h[1] * {N_INST}.0 / simds / cyc, (h[0] + h[1]) * {N_INST}.0 / simds / cyc,
         cyc, cyc / (double)h[3] * 100.0);
  fflush(stdout);
}}
int main(int argc, char** argv) {{
  const uint64_t budget = (argc > 1 ? strtoull(argv[1], 0, 10) : 20000) * 100;  // us -> 100-MHz ticks
  hipDeviceProp_t p; hipGetDeviceProperties(&p, 0);
  const int cus = p.multiProcessorCount;
  run("warm", k_XX, budget, cus);
{runs}
  return 0;
}}
"""


if __name__ == "__main__":
    if sys.argv[1] == "build":
        os.makedirs(os.path.dirname(SRC), exist_ok=True)
        open(SRC, "w").write(gen())
        subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "--offload-arch=gfx950", "-o", BIN, SRC], check=True)
        print("built", BIN)
