#!/usr/bin/env python3
"""Instruction mix per basic block of one kernel in a --save-temps .s file.

    python scripts/isa_stats.py file.s KERNEL_SYMBOL [--min N]

Prints, per basic block with at least N instructions, the counts of VALU,
LDS (ds_*), global/buffer memory, SALU and AGPR moves, and marks loop
blocks (a branch back to an earlier label).
"""
import re
import sys


def main():
    path, sym = sys.argv[1], sys.argv[2]
    mn = int(sys.argv[sys.argv.index("--min") + 1]) if "--min" in sys.argv \
        else 40
    lines = open(path).read().splitlines()
    start = next(i for i, l in enumerate(lines) if l.startswith(sym + ":"))
    end = next(i for i in range(start + 1, len(lines))
               if lines[i].strip().startswith(".Lfunc_end"))
    blocks, cur, order = {}, "entry", ["entry"]
    blocks[cur] = []
    for l in lines[start + 1:end]:
        m = re.match(r"^(\.LBB\w+):", l)
        if m:
            cur = m.group(1)
            order.append(cur)
            blocks[cur] = []
            continue
        s = l.strip()
        if not s or s.startswith(";") or s.startswith("."):
            continue
        blocks[cur].append(s.split(";")[0].strip())
    pos = {b: i for i, b in enumerate(order)}
    tot = {}
    for b in order:
        ins = blocks[b]
        c = {"valu": 0, "lds": 0, "vmem": 0, "salu": 0, "acc": 0,
             "wait": 0}
        loop = False
        for s in ins:
            op = s.split()[0]
            if op.startswith("v_accvgpr"):
                c["acc"] += 1
            elif op.startswith("v_"):
                c["valu"] += 1
            elif op.startswith("ds_"):
                c["lds"] += 1
            elif op.startswith(("global_", "buffer_", "flat_", "scratch_")):
                c["vmem"] += 1
            elif op.startswith("s_waitcnt"):
                c["wait"] += 1
            elif op.startswith("s_"):
                c["salu"] += 1
            m = re.match(r"s_cbranch\w*\s+(\.LBB\w+)|s_branch\s+(\.LBB\w+)",
                         s)
            if m:
                t = m.group(1) or m.group(2)
                if t in pos and pos[t] <= pos[b]:
                    loop = True
        for k, v in c.items():
            tot[k] = tot.get(k, 0) + v
        if len(ins) >= mn:
            print("%-16s n=%5d %s%s" % (b, len(ins), " ".join(
                "%s=%d" % kv for kv in c.items()), "  LOOP" if loop else ""))
    print("TOTAL", " ".join("%s=%d" % kv for kv in tot.items()))


if __name__ == "__main__":
    main()
