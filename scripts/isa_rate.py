#!/usr/bin/env python3
"""Steady-loop VALU issue classes of the crypto kernels under a set of
compile flags (A/B of instruction-selection knobs before a GPU run).

    python scripts/isa_rate.py [-DKNOB=V ...]

Classes from the measured gfx950 issue rates (profiles/r03_ubench_ops.txt):
full-rate VALU (v_xor/or/and/add/mov/not/lshrrev_b32, v_ashrrev,
v_lshlrev_b16/v_lshrrev_b16, v_bitop3 -- all without an SGPR operand),
half-rate VALU (everything else, and any VALU op reading an SGPR), LDS.
The issue estimate weights them by the measured chip-wide lane-op rates
(8 waves/SIMD): full 60, half 36.5, ds_read_b32 16.5 T lane-ops/s.
"""
import collections
import os
import re
import subprocess
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import isa_mix as M  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FAST = {"v_xor_b32", "v_or_b32", "v_and_b32", "v_add_u32", "v_sub_u32",
        "v_subrev_u32", "v_mov_b32", "v_not_b32", "v_lshrrev_b32",
        "v_ashrrev_i32", "v_lshlrev_b16", "v_lshrrev_b16", "v_bitop3_b32"}
RATE = {"fast": 60.0, "slow": 36.5, "lds": 16.5}


def cls(ins):
    parts = ins.split(None, 1)
    op, args = parts[0], parts[1] if len(parts) > 1 else ""
    base = re.sub(r"_e(32|64)$", "", op)
    if op.startswith("ds_"):
        return "lds", op
    if not op.startswith("v_") or op.startswith(("v_readfirstlane",
                                                  "v_readlane",
                                                  "v_writelane")):
        return "other", op
    sgpr = re.search(r"(?<![a-z_])s\[?\d", args) is not None
    if base in FAST and not sgpr:
        return "fast", op
    return "slow", base + (":s" if sgpr else "")


def main():
    flags = sys.argv[1:]
    tmp = tempfile.mkdtemp()
    for tu, kern in (("ctr10a.hip", "k_ctr_fast_any"),
                     ("ctr10a.hip", "k_ctr_fast_mk"),
                     ("gcm.hip", "k_gcmu")):
        s = os.path.join(tmp, tu + ".s")
        if not os.path.exists(s):
            subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17",
                            "--offload-arch=gfx950", "--cuda-device-only",
                            "-S", "-I" + os.path.join(ROOT, "include"),
                            "-I" + os.path.join(ROOT, "re_amd", "csrc")] +
                           flags + [os.path.join(ROOT, "re_amd", "csrc",
                                                 "hip", tu), "-o", s],
                           check=True, capture_output=True)
        lines = open(s).read().splitlines()
        for i, ln in enumerate(lines):
            m = re.match(r"^(_Z\w+):", ln)
            if not m or kern not in m.group(1):
                continue
            end = next(j for j in range(i + 1, len(lines))
                       if lines[j].strip().startswith(".Lfunc_end"))
            bl, loops = M.blocks(lines, i, end)
            if not loops:
                continue
            big = max(loops, key=lambda b: len(bl[b]))
            c = collections.Counter()
            slow = collections.Counter()
            for x in bl[big]:
                k, op = cls(x)
                c[k] += 1
                if k == "slow":
                    slow[op] += 1
            valu = c["fast"] / RATE["fast"] + c["slow"] / RATE["slow"]
            lds = c["lds"] / RATE["lds"]
            print("%-22s fast %4d slow %4d lds %4d other %4d | valu %.1f "
                  "lds %.1f (lane-ps/chunk)" % (M.short(m.group(1)),
                                                c["fast"], c["slow"],
                                                c["lds"], c["other"], valu,
                                                lds))
            print("    " + ", ".join("%s %d" % kv
                                     for kv in slow.most_common(8)))


if __name__ == "__main__":
    main()
