"""Variants of the production hash stream with independent v_mov_b32 fillers inserted at
half-rate -> full-rate transitions (does a mov, which issues free beside v_alignbit_b32, absorb the
SIMD's transition penalty?).  Writes build/ab2/<variant>.inc for tools/valu_mix2.py MIX_STREAMS."""
import os
import re
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
HALF = ("v_lshl_add_u64", "v_alignbit_b32")


def main():
    src = open(os.path.join(ROOT, "nano-dpow_amd", "csrc", "npow_hash_asm.inc")).read()
    head, rest = src.split("  asm(\n", 1)
    body, tail = rest.split("      : [value_lo]", 1)
    lines = re.findall(r'      "(.*?)\\n"\n', body)
    variants = {
        "mov64_after_hf": lambda cur, nxt: (["v_mov_b32_e64 v54, v55"]
                                            if cur.startswith(HALF) and nxt and not nxt.startswith(HALF) else []),
        "mov2_after_hf": lambda cur, nxt: (["v_mov_b32 v54, v55", "v_mov_b32 v55, v54"]
                                           if cur.startswith(HALF) and nxt and not nxt.startswith(HALF) else []),
        "mov64_after_h": lambda cur, nxt: (["v_mov_b32_e64 v54, v55"] if cur.startswith(HALF) else []),
    }
    os.makedirs(os.path.join(ROOT, "build", "ab2"), exist_ok=True)
    for name, fn in variants.items():
        out = []
        for i, ln in enumerate(lines):
            out.append(ln)
            nxt = lines[i + 1] if i + 1 < len(lines) else None
            out.extend(fn(ln, nxt))
        txt = head + "  asm(\n" + "".join(f'      "{ln}\\n"\n' for ln in out) + "      : [value_lo]" + tail
        path = os.path.join(ROOT, "build", "ab2", f"{name}.inc")
        open(path, "w").write(txt)
        print(name, len(out) - len(lines), "movs ->", path)


if __name__ == "__main__":
    sys.exit(main())
