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
              SQ_INSTS_VALU x 64 lanes x (f_fast / R_fast + f_slow /
              R_slow): f = the steady loop's full-rate / half-rate VALU
              shares (profiles/r03_isa_mix.json "classes",
              scripts/isa_mix.py), R = the chip-wide lane-op rates of the
              two classes measured at 8 waves/SIMD (medians over the
              instruction forms of scripts/ubench_ops.hip,
              profiles/r03_ubench_ops.txt)
  lds_floor_frac = SQ_INSTS_LDS x 64 x (f_b32 + 4 f_b128) / R_lds over the
              duration, R_lds the conflict-free ds_read_b32 rate
              (profiles/r03_ubench_sdwa.txt lds_fast, 8 waves/SIMD)
  issue_frac = int_frac + lds_floor_frac (the two measured kernels run
              close to the SUM of the floors, not their maximum)
  lds_frac  = SQ_LDS_IDX_ACTIVE / (GRBM_GUI_ACTIVE / 8 x 256 CUs)
"""
import csv
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SIMDS = 1024
CRYPTO = ("k_ctr_fast_any", "k_ctr_fast_mk", "k_ctr_fast_rtcp", "k_ctr_hmac",
          "k_gcm")
FAST_FORMS = ("xor_vv", "xor_kv", "and_kv", "add_kv", "mov_v", "not_v",
              "lshr_vv", "ashr_8", "lshl_b16", "lshr_b16", "add_vv_e64",
              "xor_vv_e64", "bitop3_vvv96", "bitop3_vvvec")


def class_rates(ops_txt, sdwa_txt):
    """chip-wide lane-ops/s of full-rate VALU, half-rate VALU, LDS b32"""
    fast, slow, lds = [], [], []
    for ln in open(ops_txt):
        f = ln.split()
        if len(f) < 2 or f[1] != "waves/SIMD=8" or f[0] in ("warm",
                                                         "cndmask"):
            continue
        t = float(re.search(r"([\d.]+) T lane-ops/s", ln).group(1))
        (fast if f[0] in FAST_FORMS else slow).append(t * 1e12)
    for ln in open(sdwa_txt):
        f = ln.split()
        if len(f) > 1 and f[0] == "lds_fast" and f[1] == "waves/SIMD=8":
            lds.append(float(re.search(r"([\d.]+) T lane-ops/s",
                                       ln).group(1)) * 1e12)
    med = lambda v: sorted(v)[len(v) // 2]
    return med(fast), med(slow), med(lds)


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
    r_fast, r_slow, r_lds = class_rates(
        os.path.join(ROOT, "profiles", "r03_ubench_ops.txt"),
        os.path.join(ROOT, "profiles", "r03_ubench_sdwa.txt"))
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
        mname = name.replace("k_ctr_fused", "k_ctr_fast_any")
        if t and "SQ_INSTS_VALU" in s and mname in mix:
            cl = mix[mname]["classes"]
            nv = cl.get("fast", 0) + cl.get("slow", 0)
            floor = s["SQ_INSTS_VALU"] * 64 * (
                cl.get("fast", 0) / nv / r_fast +
                cl.get("slow", 0) / nv / r_slow)
            e.update(valu_floor_s=floor, kernel_s=t, int_frac=floor / t,
                     valu_insts=s["SQ_INSTS_VALU"],
                     rates_T={"fast": r_fast / 1e12, "slow": r_slow / 1e12,
                              "lds_b32": r_lds / 1e12})
            if "SQ_INSTS_LDS" in s:
                nl = cl.get("lds", 0) + cl.get("lds_b128", 0)
                w = (cl.get("lds", 0) + 4 * cl.get("lds_b128", 0)) / nl \
                    if nl else 1.0
                lf = s["SQ_INSTS_LDS"] * 64 * w / r_lds
                e.update(lds_floor_s=lf, lds_floor_frac=lf / t,
                         issue_frac=(floor + lf) / t)
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
