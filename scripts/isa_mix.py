#!/usr/bin/env python3
"""Steady-loop instruction mix of the crypto kernels (gfx950 assembly).

    python scripts/isa_mix.py OUT.json

Compiles the kernel translation units to assembly (hipcc --cuda-device-only
-S, the product's flags), finds each kernel's largest loop block (the
steady 64-byte chunk) and records its opcode histogram.  scripts/pmc_r03.py
weights the measured per-opcode issue rates (scripts/ubench_valu.hip) by
this mix to get each kernel's VALU issue floor.  Each
instruction is also classed by its measured gfx950 issue rate
(scripts/ubench_ops.hip, profiles/r03_ubench_ops.txt): "fast" (full-rate
VALU: v_xor/or/and/add/sub/mov/not/lshrrev_b32, v_ashrrev, v_lshlrev_b16,
v_lshrrev_b16, v_bitop3 -- without an SGPR operand), "slow" (every other
VALU op, and any VALU op reading an SGPR), "lds" (ds_read/ds_write),
"lds_b128" (16-byte LDS reads, 4x the bytes).
"""
import collections
import json
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TUS = {"ctr10a.hip": ["k_ctr_fast_any", "k_ctr_fast_mk", "k_ctr_fast_rtcp",
                      "k_ctr_hmac_any"],
       "ctr14a.hip": ["k_ctr_fast_any"],
       "gcm.hip": ["k_gcmu", "k_gcm"]}


def short(sym):
    """mangled kernel symbol -> bench/profiling name "name<nr,prot>" """
    dem = subprocess.run(["c++filt", sym], capture_output=True,
                         text=True).stdout.strip()
    m = re.match(r"void (\w+)<([^>]*)>", dem)
    name, args = m.group(1), [a.strip() for a in m.group(2).split(",")]
    nr = int(args[0])
    if name == "k_ctr_hmac":
        prot, comp, uni = args[2], args[3], args[4]
        name += "" if comp == "false" else ("_uni" if uni == "true"
                                            else "_compact")
    elif name == "k_ctr_hmac_any":
        prot = args[1]
        name += "_uni" if args[2] == "true" else ""
    elif name == "k_gcm":
        prot = args[1]
        name += "_compact" if args[2] == "true" else ""
    else:
        prot = args[1]
    return "%s<%d,%d>" % (name, nr, 1 if prot == "true" else 0)


FAST = {"v_xor_b32", "v_or_b32", "v_and_b32", "v_add_u32", "v_sub_u32",
        "v_subrev_u32", "v_mov_b32", "v_not_b32", "v_lshrrev_b32",
        "v_ashrrev_i32", "v_lshlrev_b16", "v_lshrrev_b16", "v_bitop3_b32"}


def iclass(ins):
    """issue class of one instruction (see the module docstring)"""
    parts = ins.split(None, 1)
    op, args = parts[0], parts[1] if len(parts) > 1 else ""
    if op.startswith("ds_"):
        return "lds_b128" if op.endswith("b128") else "lds"
    if not op.startswith("v_") or op.startswith(("v_readfirstlane",
                                                  "v_readlane",
                                                  "v_writelane")):
        return "other"
    base = re.sub(r"_e(32|64)$", "", op)
    sgpr = re.search(r"(?<![a-z_])s\[?\d", args) is not None
    return "fast" if base in FAST and not sgpr else "slow"


def blocks(lines, start, end):
    cur, order, bl = "entry", ["entry"], {"entry": []}
    for ln in lines[start + 1:end]:
        m = re.match(r"^(\.LBB\w+):", ln)
        if m:
            cur = m.group(1)
            order.append(cur)
            bl[cur] = []
            continue
        s = ln.strip()
        if not s or s.startswith((";", ".")):
            continue
        bl[cur].append(s.split(";")[0].strip())
    pos = {b: i for i, b in enumerate(order)}
    loops = []
    for b in order:
        for s in bl[b]:
            m = re.match(r"s_c?branch\w*\s+(\.LBB\w+)", s)
            if m and m.group(1) in pos and pos[m.group(1)] <= pos[b]:
                loops.append(b)
                break
    return bl, loops


def main():
    out = sys.argv[1]
    res = {}
    tmp = tempfile.mkdtemp()
    for tu, kernels in TUS.items():
        s = os.path.join(tmp, tu + ".s")
        subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17",
                        "--offload-arch=gfx950", "--cuda-device-only", "-S",
                        "-I" + os.path.join(ROOT, "include"),
                        "-I" + os.path.join(ROOT, "re_amd", "csrc"),
                        os.path.join(ROOT, "re_amd", "csrc", "hip", tu),
                        "-o", s], check=True, capture_output=True)
        lines = open(s).read().splitlines()
        for i, ln in enumerate(lines):
            m = re.match(r"^(_Z\w+):", ln)
            if not m or not any(k in m.group(1) for k in kernels):
                continue
            sym = m.group(1)
            end = next(j for j in range(i + 1, len(lines))
                       if lines[j].strip().startswith(".Lfunc_end"))
            bl, loops = blocks(lines, i, end)
            if not loops:
                continue
            big = max(loops, key=lambda b: len(bl[b]))
            ops = collections.Counter(x.split()[0] for x in bl[big])
            cl = collections.Counter(iclass(x) for x in bl[big])
            res[short(sym)] = {"block": big, "n": len(bl[big]),
                               "ops": dict(ops.most_common()),
                               "classes": dict(cl)}
    json.dump(res, open(out, "w"), indent=1, sort_keys=True)
    for k, v in sorted(res.items()):
        print(k, v["n"])


if __name__ == "__main__":
    main()
