#!/usr/bin/env python3
"""Instruction census of the search kernel's hot loop in the built libnanopow.so (CPU only).

Unbundles the gfx950 code object, disassembles one kernel (default npow_pool_kernel_ls2_arg<false>)
and finds its hash loop: the backward branch whose body holds the generated stream (the block with
the most v_alignbit_b32).  Prints the loop's instruction counts by class, and the counts besides the
stream's own (tools/gen_hash_asm.py header: VALU per nonce), so a change to the loop's bookkeeping can
be checked before it goes to the GPU (5 non-hash VALU instructions per iteration).

    python tools/kernel_loop_census.py [--kernel SUBSTRING] [--lib PATH] [--json]
"""
import argparse
import collections
import json
import os
import re
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
LLVM = "/opt/rocm/lib/llvm/bin"
STREAM_INC = os.path.join(ROOT, "nano-dpow_amd", "csrc", "npow_hash_asm_lockstep_ld.inc")


def code_object(lib, tmp):
    fat, co = os.path.join(tmp, "fat.bin"), os.path.join(tmp, "k.co")
    subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", lib, os.path.join(tmp, "lib.tmp")],
                   check=True, capture_output=True)
    subprocess.run([f"{LLVM}/clang-offload-bundler", "--type=o", "--targets=hipv4-amdgcn-amd-amdhsa--gfx950",
                    f"--input={fat}", f"--output={co}", "--unbundle"], check=True, capture_output=True)
    return co


def disassemble(co, kernel_sub):
    out = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "-C", "--no-show-raw-insn", "--mcpu=gfx950", co],
                         check=True, capture_output=True, text=True).stdout
    funcs = re.split(r"\n(?=[0-9a-f]+ <)", out)
    for f in funcs:
        m = re.match(r"[0-9a-f]+ <(.+)>:", f)
        name = m.group(1) if m else ""
        if kernel_sub in name and not name.endswith(".kd"):
            base = int(f.split(" ", 1)[0], 16)
            insts = []
            for ln in f.splitlines()[1:]:
                m = re.match(r"\s+(\S+)(.*?)\s*//\s*([0-9A-F]+):(.*)$", ln)
                if m:
                    insts.append((int(m.group(3), 16), m.group(1), m.group(2).strip() + " " + m.group(4).strip()))
            return name, base, insts
    raise SystemExit(f"no kernel matching {kernel_sub!r}")


def klass(op):
    if op.startswith("v_"):
        return "valu"
    if op.startswith(("s_load", "s_buffer_load")):
        return "smem"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("s_cbranch", "s_branch")):
        return "branch"
    if op in ("s_waitcnt", "s_barrier", "s_setprio", "s_nop", "s_sleep"):
        return op
    return "salu"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kernel", default="npow_pool_kernel_ls2_arg<false>")
    ap.add_argument("--lib", default=os.path.join(ROOT, "nano-dpow_amd", "nanopow", "libnanopow.so"))
    ap.add_argument("--json", action="store_true")
    ap.add_argument("--dump", action="store_true", help="print the loop's instructions besides the hash stream")
    a = ap.parse_args()
    with tempfile.TemporaryDirectory() as tmp:
        name, base, insts = disassemble(code_object(a.lib, tmp), a.kernel)
    addr_idx = {ad: i for i, (ad, _, _) in enumerate(insts)}
    best = None
    for i, (ad, op, args) in enumerate(insts):
        if op.startswith(("s_cbranch", "s_branch")):
            m = re.search(r"\+0x([0-9a-f]+)>\s*$", args)
            tgt = None
            if m and base + int(m.group(1), 16) in addr_idx and base + int(m.group(1), 16) <= ad:
                tgt = base + int(m.group(1), 16)
            if tgt is None:
                continue
            body = insts[addr_idx[tgt]:i + 1]
            aligns = sum(1 for _, o, _ in body if o == "v_alignbit_b32")
            if best is None or aligns > best[0] or (aligns == best[0] and len(body) < len(best[1])):
                best = (aligns, body)
    if not best or best[0] == 0:
        raise SystemExit("no loop holding the hash stream found")
    body = best[1]
    cnt = collections.Counter(klass(op) for _, op, _ in body)
    valu_ops = collections.Counter(op for _, op, _ in body if op.startswith("v_"))
    head = open(STREAM_INC).read(2000)
    m = re.search(r"Per nonce: (\d+) VALU instructions", head)
    stream_valu = int(m.group(1)) if m else None
    res = {"kernel": name, "loop_instructions": len(body), "by_class": dict(cnt),
           "stream_valu": stream_valu, "loop_valu_besides_stream": cnt["valu"] - (stream_valu or 0),
           "non_stream_valu": sorted(((o, c) for o, c in valu_ops.items()
                                      if o not in ("v_xor_b32_e64", "v_xor_b32", "v_xor_b32_e32", "v_alignbit_b32",
                                                   "v_lshl_add_u64", "v_bitop3_b32")), key=lambda x: -x[1])}
    if a.dump:
        stream_ops = ("v_xor_b32_e64", "v_xor_b32", "v_xor_b32_e32", "v_alignbit_b32", "v_lshl_add_u64",
                      "v_bitop3_b32", "s_setprio")
        for k, (ad, op, args) in enumerate(body):
            if op not in stream_ops:
                print(f"{k:5d} {ad - base:#07x} {op} {args}")
    if a.json:
        print(json.dumps(res))
    else:
        for k, v in res.items():
            print(f"{k}: {v}")


if __name__ == "__main__":
    sys.exit(main())
