#!/usr/bin/env python3
"""VALU mixing microbenchmark for gfx950: what does an instruction cost next to another kind?

Each pattern is a sequence of instruction KINDS (xor = v_xor_b32_e64, xor2 = VOP2 v_xor_b32,
align = v_alignbit_b32, add64 = v_lshl_add_u64, lshr, addu = v_add_u32, mov, perm, bitop3);
the kernel issues it with every instruction independent of every other (destinations rotate
over v8..v39, sources are read-only v40..v63), 8 waves per SIMD, and reports SIMD cycles per
instruction from the in-kernel clock.  Writes tools/valu_mix.hip and builds build/valu_mix.
"""
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)

PATTERNS_ALL = {
    "xor": ["xor"],
    "align": ["align"],
    "add64": ["add64"],
    "xor|align alt": ["xor", "align"],
    "xor2|align alt": ["xor2", "align"],
    "xor xor|align align": ["xor", "xor", "align", "align"],
    "xor x4|align x4": ["xor"] * 4 + ["align"] * 4,
    "xor x8|align x8": ["xor"] * 8 + ["align"] * 8,
    "xor|add64 alt": ["xor", "add64"],
    "xor2|add64 alt": ["xor2", "add64"],
    "xor xor|add64": ["xor", "xor", "add64"],
    "align|add64 alt": ["align", "add64"],
    "lshr|align alt": ["lshr", "align"],
    "addu|align alt": ["addu", "align"],
    "mov|align alt": ["mov", "align"],
    "bitop3|align alt": ["bitop3", "align"],
    "xor|perm alt": ["xor", "perm"],
    "lshr|add64 alt": ["lshr", "add64"],
    "G-like mix": ["xor", "xor", "align", "align", "add64", "xor", "xor", "add64", "xor", "xor", "align", "align",
                   "add64", "xor", "xor", "lshr", "add64", "add64"],
    "G-like grouped": ["xor", "xor", "xor", "xor", "xor", "xor", "xor", "xor", "lshr", "align", "align", "align",
                       "align", "add64", "add64", "add64", "add64", "add64"],
}
PATTERNS_SDWA = {
    "mov": ["mov"],
    "movsdwa": ["movsdwa"],
    "mov|align alt": ["mov", "align"],
    "movsdwa|align alt": ["movsdwa", "align"],
    "movsdwa|add64 alt": ["movsdwa", "add64"],
    "mov|add64 alt": ["mov", "add64"],
    "mov|xor alt": ["mov", "xor"],
    "not|align alt": ["not", "align"],
    "mov64|align alt": ["mov64", "align"],
    "movdpp|align alt": ["movdpp", "align"],
    "xorsdwa|align alt": ["xorsdwa", "align"],
    "lshr movsdwa|align align": ["lshr", "movsdwa", "align", "align"],
    "G rot16 by align": ["xor", "xor", "align", "align", "add64", "xor", "xor", "add64", "xor", "xor", "align", "align",
                         "add64", "xor", "xor", "lshr", "add64", "add64"],
    "G rot16 by lshr+movsdwa": ["xor", "xor", "align", "align", "add64", "xor", "xor", "add64", "xor", "xor", "lshr",
                                "movsdwa", "lshr", "movsdwa", "add64", "xor", "xor", "lshr", "add64", "add64"],
    "G rot16 by mov-pair (upper bound)": ["xor", "xor", "align", "align", "add64", "xor", "xor", "add64", "xor", "xor",
                                          "lshr", "mov", "lshr", "mov", "add64", "xor", "xor", "lshr", "add64", "add64"],
}
import os as _os
PATTERNS = PATTERNS_SDWA if _os.environ.get("MIX_SET") == "sdwa" else PATTERNS_ALL


def emit(kind, i):
    d = 8 + (i * 2) % 32           # even destination (pairs for add64)
    s0 = 40 + (i * 2) % 12         # even sources in v40..v51
    s1 = 52 + (i * 2) % 12         # even sources in v52..v63
    if kind == "xor":
        return f"v_xor_b32_e64 v{d}, v{s0}, v{s1}"
    if kind == "xor2":
        return f"v_xor_b32 v{d}, v{s0}, v{s1}"
    if kind == "align":
        return f"v_alignbit_b32 v{d}, v{s0}, v{s1}, 24"
    if kind == "add64":
        return f"v_lshl_add_u64 v[{d}:{d + 1}], v[{s0}:{s0 + 1}], 0, v[{s1}:{s1 + 1}]"
    if kind == "lshr":
        return f"v_lshrrev_b32 v{d}, 31, v{s0}"
    if kind == "addu":
        return f"v_add_u32 v{d}, v{s0}, v{s1}"
    if kind == "mov":
        return f"v_mov_b32 v{d}, v{s0}"
    if kind == "perm":
        return f"v_perm_b32 v{d}, v{s0}, v{s1}, v{s1 + 1}"
    if kind == "movsdwa":
        return f"v_mov_b32_sdwa v{d}, v{s0} dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0"
    if kind == "xorsdwa":
        return f"v_xor_b32_sdwa v{d}, v{s0}, v{s1} dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0"
    if kind == "not":
        return f"v_not_b32 v{d}, v{s0}"
    if kind == "mov64":
        return f"v_mov_b64 v[{d}:{d + 1}], v[{s0}:{s0 + 1}]"
    if kind == "movdpp":
        return f"v_mov_b32_dpp v{d}, v{s0} quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf"
    if kind == "bitop3":
        return f"v_bitop3_b32 v{d}, v{s0}, v{s1}, v{s1 + 1} bitop3:0x96"
    raise ValueError(kind)


def main():
    n_body = 360  # instructions per asm block (a multiple of every pattern length used: 1,2,3,4,18,20)
    kernels, runs, names = [], [], []
    clob = ", ".join(f'"v{r}"' for r in range(8, 64))
    for k, (name, pat) in enumerate(PATTERNS.items()):
        lines = [emit(pat[i % len(pat)], i) for i in range(n_body)]
        asm = "\\n\\t".join(lines)
        kernels.append(f'''
__global__ __launch_bounds__(256) void mix_{k}(int iters, unsigned long long* clk) {{
  asm volatile("v_mov_b32 v40, v0\\n\\tv_mov_b32 v52, v0" ::: {clob});
  unsigned long long t0 = 0, r0 = 0;
  if (threadIdx.x == 0 && blockIdx.x == 0) {{ t0 = __builtin_amdgcn_s_memtime(); r0 = __builtin_amdgcn_s_memrealtime(); }}
  for (int it = 0; it < iters; ++it) {{
    asm volatile("{asm}" ::: {clob});
  }}
  if (threadIdx.x == 0 && blockIdx.x == 0) {{ clk[0] = __builtin_amdgcn_s_memtime() - t0; clk[1] = __builtin_amdgcn_s_memrealtime() - r0; }}
}}''')
        runs.append(f'  run(mix_{k}, "{name}", {n_body}, cus, d_clk, iters);')
    src = f'''// GENERATED by tools/valu_mix.py -- VALU mixing microbenchmark (gfx950)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#define CHECK(x) do {{ hipError_t e = (x); if (e != hipSuccess) {{ fprintf(stderr, "%s\\n", hipGetErrorString(e)); exit(1); }} }} while (0)
{"".join(kernels)}

template <class K>
static void run(K kern, const char* name, int n_body, int cus, unsigned long long* d_clk, int iters) {{
  const int blocks = cus * 8, threads = 256, reps = 3;
  kern<<<blocks, threads>>>(iters, d_clk);
  CHECK(hipDeviceSynchronize());
  hipEvent_t a, b; CHECK(hipEventCreate(&a)); CHECK(hipEventCreate(&b));
  CHECK(hipEventRecord(a));
  for (int r = 0; r < reps; ++r) kern<<<blocks, threads>>>(iters, d_clk);
  CHECK(hipEventRecord(b)); CHECK(hipEventSynchronize(b));
  float ms; CHECK(hipEventElapsedTime(&ms, a, b));
  unsigned long long clk[2]; CHECK(hipMemcpy(clk, d_clk, 16, hipMemcpyDeviceToHost));
  const double ghz = (double)clk[0] / (double)clk[1] * 0.1;
  const double ins = (double)blocks * (threads / 64) * iters * n_body * reps;
  const double simd_cycles = ms * 1e-3 * ghz * 1e9 * cus * 4;
  printf("{{\\"pattern\\": \\"%s\\", \\"clock_ghz\\": %.3f, \\"cycles_per_ins\\": %.3f}}\\n", name, ghz, simd_cycles / ins);
}}

int main(int argc, char** argv) {{
  const int iters = argc > 1 ? atoi(argv[1]) : 2048;
  hipDeviceProp_t p; CHECK(hipGetDeviceProperties(&p, 0));
  const int cus = p.multiProcessorCount;
  unsigned long long* d_clk; CHECK(hipMalloc(&d_clk, 16));
  for (int rep = 0; rep < 2; ++rep) {{
{chr(10).join(runs)}
  }}
  return 0;
}}
'''
    path = os.path.join(HERE, "valu_mix.hip")
    with open(path, "w") as f:
        f.write(src)
    os.makedirs(os.path.join(ROOT, "build"), exist_ok=True)
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-o", os.path.join(ROOT, "build", "valu_mix"),
                    path], check=True)


if __name__ == "__main__":
    main()
