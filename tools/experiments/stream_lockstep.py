#!/usr/bin/env python3
"""SIMD cycles per hash of generated hash streams in a one-workgroup-per-CU harness (1,024 lanes =
4 waves per SIMD, all of one workgroup): the production `seq` stream against `--sched lockstep`
streams, whose s_barriers keep a SIMD's waves in the same phase.  Every wave runs the same fixed
number of hash iterations (a barrier-carrying stream requires it), and the loop is timed from the
first to the last wave (s_memtime around __syncthreads), so no variant has a tail.

A pair spec `name=x.inc+y.inc@B` runs stream x on the waves whose wave-index bit B is 0 and y on
the others (both must carry the same number of barriers): the in-phase stream beside the
anti-phase one (gen_hash_asm.py --shift).

Usage: python3 tools/experiments/stream_lockstep.py name=path.inc ... -> build/stream_lockstep_g<GROUPS>
(run it on the GPU box; prints one JSON line per stream)."""
import os
import re
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
ITERS = int(os.environ.get("LOCKSTEP_ITERS", "400"))
# LOCKSTEP_GROUPS=2: two 1,024-lane workgroups per CU (8 waves per SIMD, two lockstep groups); the
# streams are then bound to v2..v63 (nonce v[6:7], value v4/v5) so the kernel fits 64 VGPRs
GROUPS = int(os.environ.get("LOCKSTEP_GROUPS", "1"))
NONCE, VLO, VHI = (6, 4, 5) if GROUPS > 1 else (100, 102, 103)
# LOCKSTEP_SKEW=P: odd workgroups first issue P dummy xors, so the two groups of a CU start out of phase
SKEW = int(os.environ.get("LOCKSTEP_SKEW", "0"))
SYNC = int(os.environ.get("LOCKSTEP_SYNC", "1"))


def bind(path):
    """The stream of an .inc with its asm operands bound to fixed registers (uniforms in s40..,
    nonce v[100:101], value v102/v103) -- values are meaningless, the issue cost is what counts."""
    txt = open(path).read()
    start = txt.index("  asm volatile(") if "  asm volatile(" in txt else txt.index("  asm(")
    asm = txt[txt.index("(", start) + 1:txt.index("      : [value_lo]")]
    out = []
    for ln in re.findall(r'"(.*?)\\n"', asm):
        ln = ln.replace("%[k8]", "s38").replace("%[k16]", "s39")
        ln = ln.replace("%[h0_lo]", "s36").replace("%[h0_hi]", "s37")
        ln = ln.replace("%[nonce_lo]", f"v{NONCE}").replace("%[nonce_hi]", f"v{NONCE + 1}")
        ln = ln.replace("%[nonce]", f"v[{NONCE}:{NONCE + 1}]").replace("%[value_lo]", f"v{VLO}").replace("%[value_hi]", f"v{VHI}")
        ln = re.sub(r"%\[u(\d+)_lo\]", lambda m: f"s{40 + 2 * int(m.group(1)) % 30}", ln)
        ln = re.sub(r"%\[u(\d+)_hi\]", lambda m: f"s{41 + 2 * int(m.group(1)) % 30}", ln)
        ln = re.sub(r"%\[u(\d+)\]", lambda m: f"s[{40 + 2 * int(m.group(1)) % 30}:{41 + 2 * int(m.group(1)) % 30}]", ln)
        out.append(ln)
    return out


def main():
    specs = [a.split("=", 1) for a in sys.argv[1:]]
    clob = ", ".join(f'"v{r}"' for r in (range(1, 64) if GROUPS > 1 else range(8, 128)))
    sclob = ", ".join(f'"s{r}"' for r in list(range(20, 32)) + list(range(36, 70))) + ', "vcc"'
    kernels, runs = [], []
    for k, (name, path) in enumerate(specs):
        bit = None
        if "@" in path:
            path, bit = path.split("@")
        paths = path.split("+")
        streams = [bind(p) for p in paths]
        lines = streams[0]
        n_valu = sum(1 for ln in lines if ln.startswith("v_"))
        n_bar = sum(1 for ln in lines if ln.startswith("s_barrier"))
        assert all(sum(1 for ln in st if ln.startswith("s_barrier")) == n_bar for st in streams), "barrier counts differ"
        asms = ["\\n\\t".join(st) for st in streams]
        # a --uload stream reads its uniforms from memory (%[up]: any readable buffer; the values do
        # not matter) into fixed SGPRs, which it clobbers
        up = "%[up]" in asms[0]
        if up:
            b0 = int(re.search(r"s_load_dwordx16 s\[(\d+):", asms[0]).group(1))
            sc = ", ".join(f'"s{r}"' for r in range(b0 - 2, b0 + 36))  # gen_hash_asm.uload_layout
            ops = f': : [up] "s"(out) : {clob}, {sc}'
        else:
            ops = f'::: {clob}, {sclob}'
        if len(asms) == 1:
            body = f'asm volatile("{asms[0]}" {ops});'
        else:
            body = (f'if ((wv >> {bit}) & 1) asm volatile("{asms[1]}" {ops});\n'
                    f'    else asm volatile("{asms[0]}" {ops});')
        # one __syncthreads per hash for a stream without barriers of its own (its waves would
        # drift apart); a lockstep stream's 96 barriers already keep them together
        skew = "\\n\\t".join(["v_xor_b32_e32 v2, v3, v2"] * max(SKEW, 1))
        # LOCKSTEP_SYNC=k (round 3): a __syncthreads after every k-th hash for a barrier-free stream
        # (0 = never; the search kernel has one per iteration)
        sync = "" if n_bar or SYNC == 0 else ("__syncthreads();" if SYNC == 1 else
                                               f"if ((it % {SYNC}) == {SYNC - 1}) __syncthreads();")
        kernels.append(f'''
__global__ __launch_bounds__(1024) void k{k}(unsigned long long* out) {{
  asm volatile("v_mov_b32 v{NONCE}, v0\\n\\tv_mov_b32 v{NONCE + 1}, 0" ::: {clob});
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  if ({SKEW} && (blockIdx.x & 1)) asm volatile("{skew}" ::: "v2", "v3");
  for (int it = 0; it < {ITERS}; ++it) {{
    {body}
    {sync}
  }}
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) {{  // per workgroup: span and CU (HW_ID cu/sh/se fields, XCC_ID)
    out[blockIdx.x * 4 + 0] = t0;
    out[blockIdx.x * 4 + 1] = t1;
    out[blockIdx.x * 4 + 2] = __builtin_amdgcn_s_getreg(4 | (31 << 11)) & 0x7f00u;
    out[blockIdx.x * 4 + 3] = __builtin_amdgcn_s_getreg(20 | (31 << 11));
  }}
}}''')
        runs.append(f'  run(k{k}, "{name}", {n_valu}, {n_bar}, cus, d);')
    src = f'''// GENERATED by tools/experiments/stream_lockstep.py
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <map>
#include <vector>
#define CHECK(x) do {{ hipError_t e = (x); if (e != hipSuccess) {{ fprintf(stderr, "%s\\n", hipGetErrorString(e)); exit(1); }} }} while (0)
{"".join(kernels)}
template <class K>
static void run(K kern, const char* name, int n_valu, int n_bar, int cus, unsigned long long* d) {{
  const int G = cus * {GROUPS};
  kern<<<G, 1024>>>(d);
  CHECK(hipDeviceSynchronize());
  kern<<<G, 1024>>>(d);
  CHECK(hipDeviceSynchronize());
  std::vector<unsigned long long> h(4 * (size_t)G);
  CHECK(hipMemcpy(h.data(), d, h.size() * 8, hipMemcpyDeviceToHost));
  // per CU (s_memtime: one counter per XCD): first start to last end over the wave-hashes each of
  // its SIMDs ran (workgroups on the CU x 4 waves per SIMD x iterations)
  std::map<std::pair<unsigned long long, unsigned long long>, std::vector<int>> cu;
  for (int g = 0; g < G; ++g) cu[{{h[4 * g + 3], h[4 * g + 2]}}].push_back(g);
  double sum = 0; int n_cu = 0, most = 0;
  for (auto& kv : cu) {{
    unsigned long long lo = ~0ull, hi = 0;
    for (int g : kv.second) {{ lo = std::min(lo, h[4 * g]); hi = std::max(hi, h[4 * g + 1]); }}
    sum += (double)(hi - lo) / ((double)kv.second.size() * 4.0 * {ITERS});
    ++n_cu; most = std::max(most, (int)kv.second.size());
  }}
  const double per_hash = sum / n_cu;  // SIMD cycles per wave-hash (64 nonces)
  printf("{{\\"stream\\": \\"%s\\", \\"groups_per_cu\\": {GROUPS}, \\"valu\\": %d, \\"barriers\\": %d, \\"cycles_per_hash\\": %.1f, \\"cycles_per_valu\\": %.3f, \\"cus\\": %d, \\"max_groups_per_cu\\": %d}}\\n",
         name, n_valu, n_bar, per_hash, per_hash / n_valu, n_cu, most);
}}
int main() {{
  hipDeviceProp_t p; CHECK(hipGetDeviceProperties(&p, 0));
  const int cus = p.multiProcessorCount;
  unsigned long long* d; CHECK(hipMalloc(&d, 4 * 8 * (size_t)cus * {GROUPS}));
{chr(10).join(runs)}
  return 0;
}}
'''
    tag = f"g{GROUPS}" + (f"s{SKEW}" if SKEW else "") + (f"y{SYNC}" if SYNC != 1 else "")
    path = os.path.join(ROOT, "build", f"stream_lockstep_{tag}.hip")
    open(path, "w").write(src)
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-o",
                    os.path.join(ROOT, "build", f"stream_lockstep_{tag}"), path], check=True)


if __name__ == "__main__":
    main()
