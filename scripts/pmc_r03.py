#!/usr/bin/env python3
"""Per-kernel PMC summary for bench.py's roofline annotations
(profiles/r03_pmc.json), keyed by the kernel's profiling name
("k_ctr_fast_any<10,1>", srtp_gpu_prof_read_named) and the workload tag
bench.py builds ("config2", "config3_rtcp", ...).

    python scripts/pmc_r03.py OUT.json WORKLOAD FETCH_DIR WRITE_DIR SQ_DIR

  traffic   = 2 x FETCH_SIZE + WRITE_SIZE, per launch (MI355X_MICROARCH.md
              HBM / rocprofv3: KiB, separate passes, gfx950 FETCH_SIZE
              reports half of a wide streaming read)
  int_frac  = the kernel's VALU issue floor / its duration.  Floor =
              SQ_INSTS_VALU / 1024 SIMDs x sum over the steady loop's
              opcode mix (profiles/r03_isa_mix.json, scripts/isa_mix.py)
              of fraction / issue rate, the rates measured per opcode at 4
              waves/SIMD (scripts/ubench_valu.hip, profiles/
              r03_ubench_valu.txt); opcodes not measured take the v_xor
              rate (the fastest: the floor is not overstated)
  lds_frac  = SQ_LDS_IDX_ACTIVE / (GRBM_GUI_ACTIVE / 8 x 256 CUs)
"""
import csv
import json
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SIMDS = 1024
CRYPTO = ("k_ctr_fast_any", "k_ctr_fast_mk", "k_ctr_hmac", "k_gcm")
# ubench_valu.hip names -> gfx950 opcodes
UB = {"xor": ["v_xor_b32_e32", "v_xor_b32_e64"],
      "add": ["v_add_u32_e32", "v_add_u32_e64"],
      "add3": ["v_add3_u32"], "perm": ["v_perm_b32"],
      "align": ["v_alignbit_b32"], "bitop3": ["v_bitop3_b32"],
      "lshl_or": ["v_lshl_or_b32"], "and_or": ["v_and_or_b32"],
      "bfe": ["v_bfe_u32"], "pk_add": ["v_pk_add_u16"],
      "lshl": ["v_lshlrev_b32_e32", "v_lshlrev_b32_e64"],
      "lshr": ["v_lshrrev_b32_e32", "v_lshrrev_b32_e64"],
      "or": ["v_or_b32_e32", "v_or_b32_e64"],
      "and": ["v_and_b32_e32", "v_and_b32_e64"],
      "dpp_mov": ["v_mov_b32_dpp"], "lshl_add": ["v_lshl_add_u32"]}


def rates(path):
    """opcode -> wave-instructions / s per SIMD at 4 waves/SIMD"""
    r = {}
    for ln in open(path):
        f = ln.split()
        if len(f) < 2 or f[1] != "waves/SIMD=4" or "[LDS]" in ln:
            continue
        t = float(re.search(r"([\d.]+) T lane-ops/s", ln).group(1))
        for op in UB.get(f[0], []):
            r[op] = t * 1e12 / (SIMDS * 64)
    return r


def short(k):
    dem = k
    m = re.match(r"void (\w+)<([^>]*)>", dem)
    if not m:
        return None
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


def counters(d):
    """kernel -> {counter: [values per launch]}, durations, grids"""
    acc, dur, grid = {}, {}, {}
    for r in csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))):
        k = r["Kernel_Name"]
        if not any(c in k for c in CRYPTO):
            continue
        v = float(r["Counter_Value"])
        acc.setdefault(k, {}).setdefault(r["Counter_Name"], []).append(v)
        grid.setdefault(k, int(r["Grid_Size"]))
        if r.get("Start_Timestamp") and r.get("End_Timestamp"):
            dur.setdefault(k, []).append(int(r["End_Timestamp"]) -
                                         int(r["Start_Timestamp"]))
    return acc, dur, grid


def main():
    out, wl, fdir, wdir, sdir = sys.argv[1:6]
    mix = json.load(open(os.path.join(ROOT, "profiles", "r03_isa_mix.json")))
    rt = rates(os.path.join(ROOT, "profiles", "r03_ubench_valu.txt"))
    xor = rt["v_xor_b32_e32"]
    fa, _, grid = counters(fdir)
    wa, _, _ = counters(wdir)
    sa, sdur, _ = counters(sdir)
    try:
        res = json.load(open(out))
    except (OSError, ValueError):
        res = {"entries": []}
    res["entries"] = [e for e in res["entries"] if e["workload"] != wl]
    for k in sorted(set(fa) | set(sa)):
        name = short(k)
        if not name:
            continue
        e = {"kernel": name, "workload": wl, "rocprof_name": k,
             "pkts_per_launch": grid.get(k)}
        f = [v for v in fa.get(k, {}).get("FETCH_SIZE", []) if v > 0]
        w = [v for v in wa.get(k, {}).get("WRITE_SIZE", []) if v > 0]
        if f and w:
            e["fetch_bytes_x2"] = 2.0 * 1024 * sum(f) / len(f)
            e["write_bytes"] = 1024.0 * sum(w) / len(w)
            e["traffic_bytes_per_launch"] = e["fetch_bytes_x2"] + \
                e["write_bytes"]
        s = {c: sum(v) / len(v) for c, v in sa.get(k, {}).items()}
        t = sorted(sdur[k])[len(sdur[k]) // 2] * 1e-9 if sdur.get(k) else 0
        if t and "SQ_INSTS_VALU" in s and name in mix:
            ops = {o: c for o, c in mix[name]["ops"].items()
                   if o.startswith("v_") and not o.startswith("v_accvgpr")}
            tot = sum(ops.values())
            per = sum(c / tot / rt.get(o, xor) for o, c in ops.items())
            floor = s["SQ_INSTS_VALU"] / SIMDS * per
            e.update(valu_floor_s=floor, kernel_s=t, int_frac=floor / t,
                     valu_insts=s["SQ_INSTS_VALU"])
        if "SQ_LDS_IDX_ACTIVE" in s and s.get("GRBM_GUI_ACTIVE"):
            e["lds_frac"] = s["SQ_LDS_IDX_ACTIVE"] / (
                s["GRBM_GUI_ACTIVE"] / 8 * 256)
            if t:
                e["clock_GHz"] = s["GRBM_GUI_ACTIVE"] / 8 / t / 1e9
        if len(e) > 4:
            res["entries"].append(e)
    json.dump(res, open(out, "w"), indent=1, sort_keys=True)
    for e in res["entries"]:
        if e["workload"] == wl:
            print(json.dumps(e))


if __name__ == "__main__":
    main()
