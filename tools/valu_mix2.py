#!/usr/bin/env python3
"""Time-bounded VALU mixing microbenchmark (gfx950): every wave repeats its instruction block
until the same wall-clock budget has passed since it started, so each SIMD stays saturated for
the whole measurement (a fixed-iteration kernel ends in a tail where VALU issue, which favours
a SIMD's oldest wave, has only one or two waves left -- DESIGN.md section 4).  Reports SIMD
cycles per instruction.  Patterns as tools/valu_mix.py, plus "real": the production hash stream.

Usage: python3 tools/valu_mix2.py [blocks_per_cu] [budget_us]  -> writes tools/valu_mix2.hip and
builds build/valu_mix2
"""
import os
import re
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, HERE)
from valu_mix import emit, PATTERNS_ALL  # noqa: E402

PATTERNS = {
    "xor": ["xor"], "xor2": ["xor2"], "align": ["align"], "add64": ["add64"], "lshr": ["lshr"],
    "mov": ["mov"], "bitop3": ["bitop3"],
    "xor|align alt": ["xor", "align"], "xor|add64 alt": ["xor", "add64"],
    "xor xor|add64": ["xor", "xor", "add64"], "align|add64 alt": ["align", "add64"],
    "mov|align alt": ["mov", "align"],
    "G-like mix": PATTERNS_ALL["G-like mix"],
    "xor xor|align align": ["xor", "xor", "align", "align"],
    "xor x4|align x4": ["xor"] * 4 + ["align"] * 4,
    "xor x8|align x8": ["xor"] * 8 + ["align"] * 8,
    "xor dep chain": ["xordep"], "align dep chain": ["aligndep"], "add64 dep chain": ["add64dep"],
    "xor dep x4 chains": ["xordep4"],
    "alignbyte": ["alignbyte"], "alignbyte2": ["alignbyte2"], "addco": ["addco"], "addc": ["addc"],
    "addco|addc": ["addco", "addc"], "addco3|addc3": ["addco3", "addc3"], "lshlor": ["lshlor"],
    "addco4|addc4 sgpr-rot": ["addco4a", "addc4a"], "addco6 sgpr-rot": ["addco8"],
    "xor xor|addco4 addc4 sgpr-rot": ["xor", "xor", "addco4b", "addc4b"],
    "xor|addco6 sgpr-rot alt": ["xor", "addco8"],
    # free fillers beside half-rate ops, and fillers at half -> full transitions (round 2)
    "mov|add64 alt": ["mov", "add64"], "mov e64|align alt": ["mov3", "align"], "not|align alt": ["not", "align"],
    "mov64|align alt": ["mov64", "align"], "movsdwa|align alt": ["movsdwa", "align"],
    "xorsdwa|align alt": ["xorsdwa", "align"], "movdpp|align alt": ["movdpp", "align"],
    "align mov xor": ["align", "mov", "xor"], "align mov e64 xor": ["align", "mov3", "xor"],
    "add64 mov xor": ["add64", "mov", "xor"], "add64 xor": ["add64", "xor"],
    "align mov mov xor": ["align", "mov", "mov", "xor"], "xor align mov": ["xor", "align", "mov"],
    # long runs of one class per wave (round 2): do waves in different phases overlap the classes?
    "xor x16|align x16": ["xor"] * 16 + ["align"] * 16, "xor x32|align x32": ["xor"] * 32 + ["align"] * 32,
    "xor x64|align x64": ["xor"] * 64 + ["align"] * 64, "xor x128|align x128": ["xor"] * 128 + ["align"] * 128,
    "xor x32|add64 x32": ["xor"] * 32 + ["add64"] * 32, "xor x64|add64 x64": ["xor"] * 64 + ["add64"] * 64,
    "x8 a8 d4 (4 G lockstep)": ["xor"] * 8 + ["align"] * 8 + ["add64"] * 4,
    "x16 a16 d8 (8 G lockstep)": ["xor"] * 16 + ["align"] * 16 + ["add64"] * 8,
    "x32 a32 d16 (16 G lockstep)": ["xor"] * 32 + ["align"] * 32 + ["add64"] * 16,
    "lshl": ["lshl"], "or": ["or"], "lshr64": ["lshr64"], "add3": ["add3"], "addu": ["addu"],
    "xor|alignbyte alt": ["xor", "alignbyte"], "xor|lshlor alt": ["xor", "lshlor"],
    "xor xor|addco addc": ["xor", "xor", "addco", "addc"],
    "G all-F (byte rot + co/c adds)": ["addco", "addc", "xor", "xor", "alignbyte", "alignbyte", "addco", "addc",
                                       "xor", "xor", "alignbyte", "alignbyte", "addco", "addc", "xor", "xor",
                                       "lshr", "lshlor", "lshr", "lshlor"],
    "add64 sgpr": ["addsgpr"],
    "mul24": ["mul24"], "mul24k": ["mul24k"], "mad24": ["mad24"], "mad24s": ["mad24s"], "mad16": ["mad16"],
    "lshl e64": ["lshlk"], "lshr24 e64": ["lshr8"],
    "xor|mad24s alt": ["xor", "mad24s"], "lshr|mad24s alt": ["lshr8", "mad24s"],
    "G rot via mad24": ["xor", "xor", "lshr8", "mad24s", "lshr8", "mad24s", "add64", "xor", "xor", "add64"],
    "G rot via align": ["xor", "xor", "align", "align", "add64", "xor", "xor", "add64"],
    "P2 mad->align": ["xor", "xor", "lshr8", "align", "lshr8", "align", "add64", "xor", "xor", "add64"],
    "P3 lshr->xor": ["xor", "xor", "xor", "mad24s", "xor", "mad24s", "add64", "xor", "xor", "add64"],
    "P4 mad->add64": ["xor", "xor", "lshr8", "add64", "lshr8", "add64", "add64", "xor", "xor", "add64"],
    "P5 lshr->xor mad->align": ["xor", "xor", "xor", "align", "xor", "align", "add64", "xor", "xor", "add64"],
    "P6 FFFHFHHFFH all xor/align": ["xor", "xor", "xor", "align", "xor", "align", "align", "xor", "xor", "align"],
    "P7 FFFHFHHFFH mad only": ["xor", "xor", "xor", "mad24s", "xor", "mad24s", "mad24s", "xor", "xor", "mad24s"],
    "P8 lshr|align alt": ["lshr8", "align"],
    "P9 lshr|add64 alt": ["lshr8", "add64"],
    "P10 lshr|mad24s": ["lshr8", "mad24s"],
    "P11 xor|mad24s": ["xor", "mad24s"],
    "P12 FFHH xor/mad": ["xor", "xor", "mad24s", "mad24s"],
    "P13 FFHH xor/align": ["xor", "xor", "align", "align"],
    "Q1 mad24s|add64": ["mad24s", "add64"], "Q2 mad24s|align": ["mad24s", "align"],
    "Q3 mad24|add64": ["mad24", "add64"], "Q4 mul24|add64": ["mul24", "add64"],
    "Q5 lshl|add64": ["lshlk", "add64"], "Q6 mad24s|add64|xor|xor": ["mad24s", "add64", "xor", "xor"],
    "Q7 align|add64|xor|xor": ["align", "add64", "xor", "xor"], "Q8 mad24s|xor|add64|xor": ["mad24s", "xor", "add64", "xor"],
    "Q9 lshl|align": ["lshlk", "align"], "Q10 mul24|align": ["mul24", "align"],
    "Q11 add64 sgpr|align": ["addsgpr", "align"], "Q12 mad24s|lshl": ["mad24s", "lshlk"],
    "mad64": ["mad64"], "mad64n": ["mad64n"], "mullo": ["mullo"], "mulhi24": ["mulhi24"],
    "mad64|align": ["mad64", "align"], "mad64|add64": ["mad64", "add64"], "mad64|xor": ["mad64", "xor"],
    "mad64n|align": ["mad64n", "align"], "mulhi24|align": ["mulhi24", "align"],
    "chain xor": ("chain", ["xor"]), "chain xor|align": ("chain", ["xor", "align"]),
    "chain xor|add64": ("chain", ["xor", "add64"]), "chain xor xor|add64": ("chain", ["xor", "xor", "add64"]),
    "chain G-like mix": ("chain", PATTERNS_ALL["G-like mix"]),
}


def emit_chain(kinds, n):
    """The kinds in order, each instruction reading the previous one's result as src0 (a
    dependent chain, as in the generated stream's `seq` order), destinations rotating over
    even registers v8..v38."""
    out, prev = [], 40
    for i in range(n):
        k = kinds[i % len(kinds)]
        d = 8 + (i * 2) % 32
        s1 = 52 + (i * 2) % 12
        if k == "xor":
            out.append(f"v_xor_b32_e64 v{d}, v{prev}, v{s1}")
        elif k == "align":
            out.append(f"v_alignbit_b32 v{d}, v{prev}, v{s1}, 24")
        elif k == "add64":
            out.append(f"v_lshl_add_u64 v[{d}:{d + 1}], v[{prev}:{prev + 1}], 0, v[{s1}:{s1 + 1}]")
        elif k == "lshr":
            out.append(f"v_lshrrev_b32_e64 v{d}, 31, v{prev}")
        else:
            raise ValueError(k)
        prev = d
    return out


def emit2(kind, i):
    """emit() plus dependent chains: every instruction reads the previous one's result
    (xordep4: four interleaved chains)."""
    if kind == "xordep":
        return "v_xor_b32_e64 v8, v8, v40"
    if kind == "xordep4":
        return f"v_xor_b32_e64 v{8 + i % 4}, v{8 + i % 4}, v40"
    if kind == "aligndep":
        return "v_alignbit_b32 v8, v8, v40, 24"
    d, s0, s1 = 8 + (i * 2) % 32, 40 + (i * 2) % 12, 52 + (i * 2) % 12
    if kind == "alignbyte":
        return f"v_alignbyte_b32 v{d}, v{s0}, v{s1}, 3"
    if kind == "alignbyte2":
        return f"v_alignbyte_b32 v{d}, v{s0}, v{s1}, 2"
    if kind == "addco":
        return f"v_add_co_u32 v{d}, vcc, v{s0}, v{s1}"
    if kind == "addc":
        return f"v_addc_co_u32 v{d + 1}, vcc, v{s0 + 1}, v{s1 + 1}, vcc"
    if kind == "addco3":
        return f"v_add_co_u32_e64 v{d}, s[20:21], v{s0}, v{s1}"
    if kind == "addc3":
        return f"v_addc_co_u32_e64 v{d + 1}, s[20:21], v{s0 + 1}, v{s1 + 1}, s[20:21]"
    if kind in ("addco4a", "addc4a", "addco4b", "addc4b"):
        # carry in an SGPR pair rotating over s[20:21]..s[26:27]: a = pattern of 2 (co, c), b = of 4
        k = 20 + 2 * ((i // (2 if kind.endswith("a") else 4)) % 4)
        if kind.startswith("addco"):
            return f"v_add_co_u32_e64 v{d}, s[{k}:{k + 1}], v{s0}, v{s1}"
        return f"v_addc_co_u32_e64 v{d + 1}, s[{k}:{k + 1}], v{s0 + 1}, v{s1 + 1}, s[{k}:{k + 1}]"
    if kind == "addco8":  # six rotating pairs, carry-out only
        k = 20 + 2 * (i % 6)
        return f"v_add_co_u32_e64 v{d}, s[{k}:{k + 1}], v{s0}, v{s1}"
    if kind == "mov3":
        return f"v_mov_b32_e64 v{d}, v{s0}"
    if kind == "lshlor":
        return f"v_lshl_or_b32 v{d}, v{s0}, 8, v{s1}"
    if kind == "lshl":
        return f"v_lshlrev_b32 v{d}, 8, v{s0}"
    if kind == "or":
        return f"v_or_b32 v{d}, v{s0}, v{s1}"
    if kind == "lshr64":
        return f"v_lshrrev_b64 v[{d}:{d + 1}], 24, v[{s0}:{s0 + 1}]"
    if kind == "add3":
        return f"v_add3_u32 v{d}, v{s0}, v{s1}, v{s1 + 1}"
    if kind == "addu":
        return f"v_add_u32 v{d}, v{s0}, v{s1}"
    if kind == "addsgpr":
        return f"v_lshl_add_u64 v[{d}:{d + 1}], v[{s0}:{s0 + 1}], 0, s[40:41]"
    if kind == "mul24":
        return f"v_mul_u32_u24_e64 v{d}, v{s0}, s40"
    if kind == "mul24k":
        return f"v_mul_u32_u24 v{d}, 0x100, v{s0}"
    if kind == "mad24":
        return f"v_mad_u32_u24 v{d}, v{s0}, 8, v{s1}"
    if kind == "mad24s":
        return f"v_mad_u32_u24 v{d}, v{s0}, s40, v{s1}"
    if kind == "mad16":
        return f"v_mad_u32_u16 v{d}, v{s0}, s40, v{s1}"
    if kind == "lshlk":
        return f"v_lshlrev_b32_e64 v{d}, 8, v{s0}"
    if kind == "lshr8":
        return f"v_lshrrev_b32_e64 v{d}, 24, v{s0}"
    if kind == "mad64":
        return f"v_mad_u64_u32 v[{d}:{d + 1}], s[20:21], v{s0}, v{s1}, v[{s1}:{s1 + 1}]"
    if kind == "mad64n":  # carry-out to a rotating SGPR pair
        return f"v_mad_u64_u32 v[{d}:{d + 1}], s[{20 + (i * 2) % 8}:{21 + (i * 2) % 8}], v{s0}, 1, v[{s1}:{s1 + 1}]"
    if kind == "mullo":
        return f"v_mul_lo_u32 v{d}, v{s0}, v{s1}"
    if kind == "mulhi24":
        return f"v_mul_hi_u32_u24_e64 v{d}, v{s0}, v{s1}"
    if kind == "add64dep":
        return "v_lshl_add_u64 v[8:9], v[8:9], 0, v[40:41]"
    return emit(kind, i)


def real_stream(path=None):
    """A generated hash stream (default: production npow_hash_asm.inc) with operands bound to
    fixed registers."""
    txt = open(path or os.path.join(ROOT, "nano-dpow_amd", "csrc", "npow_hash_asm.inc")).read()
    asm = txt[txt.index("  asm(") + 6:txt.index("      : [value_lo]")]
    out = []
    for ln in re.findall(r'"(.*?)\\n"', asm):
        ln = ln.replace("%[k8]", "s38").replace("%[k16]", "s39")
        ln = ln.replace("%[h0_lo]", "s36").replace("%[h0_hi]", "s37")
        ln = ln.replace("%[nonce_lo]", "v56").replace("%[nonce_hi]", "v57")
        ln = ln.replace("%[nonce]", "v[56:57]").replace("%[value_lo]", "v58").replace("%[value_hi]", "v59")
        ln = re.sub(r"%\[u(\d+)_lo\]", lambda m: f"s{40 + 2 * int(m.group(1)) % 30}", ln)
        ln = re.sub(r"%\[u(\d+)_hi\]", lambda m: f"s{41 + 2 * int(m.group(1)) % 30}", ln)
        ln = re.sub(r"%\[u(\d+)\]", lambda m: f"s[{40 + 2 * int(m.group(1)) % 30}:{41 + 2 * int(m.group(1)) % 30}]", ln)
        out.append(ln)
    return out


def main():
    bpc = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    budget_us = int(sys.argv[2]) if len(sys.argv) > 2 else 5000
    n_body = int(os.environ.get("MIX_NBODY", "360"))
    clob = ", ".join(f'"v{r}"' for r in range(8, 64))
    sclob = ", ".join(f'"s{r}"' for r in range(36, 70))
    cclob = ", ".join(f'"s{r}"' for r in range(20, 32))  # carry pairs of the SGPR-carry patterns / streams
    kernels, runs = [], []
    items = list(PATTERNS.items()) + [("real hash stream", None)]
    # extra generated streams: MIX_STREAMS="name=path.inc,name2=path2.inc"
    for spec in filter(None, os.environ.get("MIX_STREAMS", "").split(",")):
        nm, path = spec.split("=", 1)
        items.append((f"stream {nm}", path))
    if os.environ.get("MIX_ONLY"):
        keep = os.environ["MIX_ONLY"].split(",")
        items = [it for it in items if it[0] in keep or it[0].startswith("stream ")]
    for k, (name, pat) in enumerate(items):
        if pat is None or isinstance(pat, str):
            lines = real_stream(pat)
        elif isinstance(pat, tuple):  # ("chain", kinds)
            lines = emit_chain(pat[1], n_body)
        else:
            lines = [emit2(pat[i % len(pat)], i) for i in range(n_body)]
        n_ins = sum(1 for ln in lines if ln.startswith("v_"))
        asm = "\\n\\t".join(lines)
        kernels.append(f'''
__global__ __launch_bounds__(256) void mix_{k}(unsigned long long* out) {{
  unsigned long long t0, now, n = 0;
  asm volatile("s_memrealtime %0\\n\\ts_waitcnt lgkmcnt(0)" : "=s"(t0) :: "memory");
  const unsigned long long m0 = __builtin_amdgcn_s_memtime();
  asm volatile("v_mov_b32 v40, v0\\n\\tv_mov_b32 v52, v0\\n\\tv_mov_b32 v56, v0\\n\\tv_mov_b32 v57, 0" ::: {clob});
  do {{
    asm volatile("{asm}" ::: {clob}, {sclob}, "vcc", {cclob});
    ++n;
    asm volatile("s_memrealtime %0\\n\\ts_waitcnt lgkmcnt(0)" : "=s"(now) :: "memory");
  }} while (now - t0 < {budget_us * 100}ull);
  if ((threadIdx.x & 63) == 0) atomicAdd(&out[0], n);
  if (threadIdx.x == 0 && blockIdx.x == 0) {{ out[1] = __builtin_amdgcn_s_memtime() - m0; out[2] = now - t0; }}
}}''')
        runs.append(f'  run(mix_{k}, "{name}", {n_ins}, cus, d_out, clk);')
    src = f'''// GENERATED by tools/valu_mix2.py -- time-bounded VALU mixing microbenchmark (gfx950)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#define CHECK(x) do {{ hipError_t e = (x); if (e != hipSuccess) {{ fprintf(stderr, "%s\\n", hipGetErrorString(e)); exit(1); }} }} while (0)
__global__ void clock_probe(unsigned long long* c) {{
  unsigned long long a = __builtin_amdgcn_s_memtime(), r = __builtin_amdgcn_s_memrealtime();
  unsigned long long x = 1;
  for (int i = 0; i < 2000000; ++i) x = x * 3 + 1;
  c[0] = __builtin_amdgcn_s_memtime() - a; c[1] = __builtin_amdgcn_s_memrealtime() - r; c[2] = x;
}}
{"".join(kernels)}

template <class K>
static void run(K kern, const char* name, int n_ins, int cus, unsigned long long* d_out, double ghz) {{
  const int blocks = cus * {bpc};
  kern<<<blocks, 256>>>(d_out);
  CHECK(hipDeviceSynchronize());
  CHECK(hipMemset(d_out, 0, 8));
  kern<<<blocks, 256>>>(d_out);
  CHECK(hipDeviceSynchronize());
  unsigned long long o[3]; CHECK(hipMemcpy(o, d_out, 24, hipMemcpyDeviceToHost));
  const unsigned long long n = o[0];
  ghz = (double)o[1] / (double)o[2] * 0.1;                       // this run's shader clock
  const double ins = (double)n * n_ins;                          // wave-instructions issued
  const double simd_cycles = {budget_us}e-6 * ghz * 1e9 * cus * 4; // SIMD-cycles in the budget
  printf("{{\\"pattern\\": \\"%s\\", \\"blocks_per_cu\\": {bpc}, \\"ins_per_block\\": %d, \\"clock_ghz\\": %.3f, \\"cycles_per_ins\\": %.3f}}\\n",
         name, n_ins, ghz, simd_cycles / ins);
}}

int main() {{
  hipDeviceProp_t p; CHECK(hipGetDeviceProperties(&p, 0));
  const int cus = p.multiProcessorCount;
  unsigned long long* d_out; CHECK(hipMalloc(&d_out, 64));
  // shader clock under load: ratio of s_memtime to the 100-MHz s_memrealtime
  clock_probe<<<cus * 4, 256>>>(d_out); CHECK(hipDeviceSynchronize());
  unsigned long long c[3]; CHECK(hipMemcpy(c, d_out, 24, hipMemcpyDeviceToHost));
  const double clk = (double)c[0] / (double)c[1] * 0.1;
  printf("{{\\"clock_ghz\\": %.3f}}\\n", clk);
{chr(10).join(runs)}
  return 0;
}}
'''
    path = os.path.join(HERE, "valu_mix2.hip")
    with open(path, "w") as f:
        f.write(src)
    os.makedirs(os.path.join(ROOT, "build"), exist_ok=True)
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-o",
                    os.path.join(ROOT, "build", f"valu_mix2_b{bpc}"), path], check=True)


if __name__ == "__main__":
    main()
