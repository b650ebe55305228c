#!/usr/bin/env python3
"""Does keeping a SIMD's waves in the same instruction phase remove the full/half-rate mixing cost?

VALU issue on a SIMD interleaves its waves, so even when every wave's own stream has long runs of
full-rate (xor) and half-rate (alignbit) instructions, the SIMD sees them mixed (DESIGN.md section 4:
runs of 1..8 cost the same).  Here one 1,024-lane workgroup per CU puts 4 waves on every SIMD, all
of one workgroup, and an s_barrier between runs keeps them in the same phase: if the mixing cost is
a SIMD-level transition cost, runs + barriers should approach the additive cost.

Kernels (fixed iteration count, every wave the same, an s_barrier closing every 128-instruction
block so no variant has a tail): R xors then R alignbits (or v_lshl_add_u64), with or without a
barrier after each run, for R = 4..64; the alternating baseline; pure streams.  Reports SIMD cycles
per instruction from s_memtime over the loop, timed to the workgroup's last wave.

Usage: python3 tools/experiments/phase_lockstep.py -> build/phase_lockstep (run it on the GPU box)
"""
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
ITERS = 2000


def run_block(kind, r, i0):
    out = []
    for i in range(r):
        d, s0, s1 = 8 + ((i0 + i) * 2) % 32, 40 + ((i0 + i) * 2) % 12, 52 + ((i0 + i) * 2) % 12
        if kind == "xor":
            out.append(f"v_xor_b32_e64 v{d}, v{s0}, v{s1}")
        elif kind == "align":
            out.append(f"v_alignbit_b32 v{d}, v{s0}, v{s1}, 24")
        else:
            out.append(f"v_lshl_add_u64 v[{d}:{d + 1}], v[{s0}:{s0 + 1}], 0, v[{s1}:{s1 + 1}]")
    return out


def body(r, barrier, hkind="align", total=128):
    lines = []
    i = 0
    while i < total:
        lines += run_block("xor", r, i)
        if barrier:
            lines.append("s_barrier")
        lines += run_block(hkind, r, i)
        if barrier:
            lines.append("s_barrier")
        i += 2 * r
    return lines


WAVES_PER_SIMD = int(os.environ.get("LOCKSTEP_WAVES", "4"))
GROUPS = int(os.environ.get("LOCKSTEP_GROUPS", "1"))  # workgroups per CU (2: two lockstep groups per SIMD)


def main():
    # every block ends in an s_barrier, so no variant has a launch tail (the waves of a SIMD finish
    # together); "+barrier" variants have one after every run as well (lockstep phases)
    blk = ["s_barrier"]
    variants = [("alternating", body(1, False) + blk), ("alternating add64", body(1, False, "add64") + blk)]
    for r in (4, 8, 16, 32, 64):
        variants.append((f"runs{r}", body(r, False) + blk))
        variants.append((f"runs{r}+barrier", body(r, True)))
        variants.append((f"runs{r}+barrier add64", body(r, True, "add64")))
    # hash-shaped intervals: C independent G chains per wave (4 G's of a half-round x nonces per lane),
    # each interval = the F-run of one G step for every chain, then the H-run of the next step,
    # then (optionally) an s_barrier.  Per G: (2F,1H) (2F,2align+1H) (2F,2align+1H) (3F,2H).
    def hashlike(c, barrier):
        lines = []
        for f, al, ad in ((2, 0, 1), (2, 2, 1), (2, 2, 1), (3, 0, 2)):
            lines += run_block("xor", f * c, 0) + run_block("align", al * c, 0) + run_block("add64", ad * c, 0)
            if barrier:
                lines.append("s_barrier")
        return lines
    for c in (4, 8, 12, 16):
        variants.append((f"hashlike C{c}+barrier", hashlike(c, True)))
        variants.append((f"hashlike C{c}", hashlike(c, False) + blk))
    # one F-run + one H-run per barrier, run length R
    for r in (8, 16, 24, 32, 48):
        variants.append((f"x{r} a{r} |barrier", run_block("xor", r, 0) + run_block("align", r, 0) + blk))
    # probes of the runs64 result
    variants.append(("runs64 x2 per barrier", body(64, False) + body(64, False) + blk))
    variants.append(("runs64 no barrier", body(64, False)))
    variants.append(("align64 then xor64", run_block("align", 64, 0) + run_block("xor", 64, 0) + blk))
    variants.append(("runs64 add64", body(64, False, "add64") + blk))
    variants.append(("runs32 x4 per barrier", body(32, False) * 1 + body(32, False) + blk))
    variants.append(("xor96 align32", run_block("xor", 96, 0) + run_block("align", 32, 0) + blk))
    variants.append(("xor32 align96", run_block("xor", 32, 0) + run_block("align", 96, 0) + blk))
    variants.append(("xor only", run_block("xor", 128, 0) + blk))
    variants.append(("align only", run_block("align", 128, 0) + blk))
    variants.append(("add64 only", run_block("add64", 128, 0) + blk))
    clob = ", ".join(f'"v{r}"' for r in range(8, 64))
    kernels, runs = [], []
    for k, (name, lines) in enumerate(variants):
        n_ins = sum(1 for ln in lines if ln.startswith("v_"))
        asm = "\\n\\t".join(lines)
        kernels.append(f'''
__global__ __launch_bounds__({256 * WAVES_PER_SIMD}) void k{k}(unsigned long long* out) {{
  asm volatile("v_mov_b32 v40, v0\\n\\tv_mov_b32 v52, v0" ::: {clob});
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < {ITERS}; ++it)
    asm volatile("{asm}" ::: {clob});
  __syncthreads();  // the workgroup's last wave, not wave 0 (issue favours the oldest wave)
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) {{  // per workgroup: span and where it ran (HW_ID cu/sh/se fields, XCC_ID)
    out[blockIdx.x * 4 + 0] = t0;
    out[blockIdx.x * 4 + 1] = t1;
    out[blockIdx.x * 4 + 2] = __builtin_amdgcn_s_getreg(4 | (31 << 11)) & 0x7f00u;  // cu_id, sh_id, se_id
    out[blockIdx.x * 4 + 3] = __builtin_amdgcn_s_getreg(20 | (31 << 11));
  }}
}}''')
        runs.append(f'  run(k{k}, "{name}", {n_ins}, cus, d);')
    src = f'''// GENERATED by tools/experiments/phase_lockstep.py
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <map>
#include <vector>
#define CHECK(x) do {{ hipError_t e = (x); if (e != hipSuccess) {{ fprintf(stderr, "%s\\n", hipGetErrorString(e)); exit(1); }} }} while (0)
{"".join(kernels)}
template <class K>
static void run(K kern, const char* name, int n_ins, int cus, unsigned long long* d) {{
  const int G = cus * {GROUPS};
  kern<<<G, {256 * WAVES_PER_SIMD}>>>(d);
  CHECK(hipDeviceSynchronize());
  kern<<<G, {256 * WAVES_PER_SIMD}>>>(d);
  CHECK(hipDeviceSynchronize());
  std::vector<unsigned long long> h(4 * (size_t)G);
  CHECK(hipMemcpy(h.data(), d, h.size() * 8, hipMemcpyDeviceToHost));
  // per CU (s_memtime is one counter per XCD): span from its first start to its last end, over
  // the instructions every SIMD of that CU issued = its workgroups x waves per SIMD x stream
  std::map<std::pair<unsigned long long, unsigned long long>, std::vector<int>> cu;
  for (int g = 0; g < G; ++g) cu[{{h[4 * g + 3], h[4 * g + 2]}}].push_back(g);
  double sum = 0; int n_cu = 0, most = 0;
  for (auto& kv : cu) {{
    unsigned long long lo = ~0ull, hi = 0;
    for (int g : kv.second) {{ lo = std::min(lo, h[4 * g]); hi = std::max(hi, h[4 * g + 1]); }}
    sum += (double)(hi - lo) / ((double)kv.second.size() * {WAVES_PER_SIMD} * n_ins * {ITERS});
    ++n_cu; most = std::max(most, (int)kv.second.size());
  }}
  printf("{{\\"variant\\": \\"%s\\", \\"ins_per_block\\": %d, \\"cycles_per_ins\\": %.3f, \\"cus\\": %d, \\"max_groups_per_cu\\": %d}}\\n",
         name, n_ins, sum / n_cu, n_cu, most);
}}
int main() {{
  hipDeviceProp_t p; CHECK(hipGetDeviceProperties(&p, 0));
  const int cus = p.multiProcessorCount;
  unsigned long long* d; CHECK(hipMalloc(&d, 4 * 8 * (size_t)cus * {GROUPS}));
{chr(10).join(runs)}
  return 0;
}}
'''
    path = os.path.join(ROOT, "build", f"phase_lockstep_w{WAVES_PER_SIMD}g{GROUPS}.hip")
    os.makedirs(os.path.dirname(path), exist_ok=True)
    open(path, "w").write(src)
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-o", os.path.join(ROOT, "build", f"phase_lockstep_w{WAVES_PER_SIMD}g{GROUPS}"),
                    path], check=True)


if __name__ == "__main__":
    main()
