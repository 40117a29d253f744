#!/usr/bin/env python3
"""Instruction-class sequence of one basic block (scheduling check).

    python scripts/isa_seq.py file.s KERNEL_SYMBOL .LBBx_y

L = ds_* (LDS), | = s_waitcnt, a = v_alignbit, p = v_perm, 3 = v_add3,
v = other VALU, G = global/buffer, S = scratch, s = other scalar.  Shows
whether the LDS lookups of the cipher overlap the SHA-1 VALU chain.
"""
import re
import sys


def main():
    path, sym, blk = sys.argv[1:4]
    lines = open(path).read().splitlines()
    s = next(i for i, l in enumerate(lines) if l.startswith(sym + ":"))
    i = next(j for j in range(s, len(lines)) if lines[j].startswith(blk + ":"))
    out = []
    for l in lines[i + 1:]:
        if re.match(r"^\.LBB", l) or l.strip().startswith(".Lfunc_end"):
            break
        t = l.strip().split()
        if not t or t[0].startswith((";", ".")):
            continue
        op = t[0]
        if op.startswith("ds_"):
            out.append("L")
        elif op.startswith("s_waitcnt"):
            out.append("|")
        elif op.startswith("v_alignbit"):
            out.append("a")
        elif op.startswith("v_perm"):
            out.append("p")
        elif op.startswith("v_add3"):
            out.append("3")
        elif op.startswith("v_"):
            out.append("v")
        elif op.startswith("scratch_"):
            out.append("S")
        elif op.startswith(("global", "buffer")):
            out.append("G")
        else:
            out.append("s")
    s = "".join(out)
    for k in range(0, len(s), 120):
        print(s[k:k + 120])


if __name__ == "__main__":
    main()
