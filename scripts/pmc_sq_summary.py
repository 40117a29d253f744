#!/usr/bin/env python3
"""Per-kernel SQ counter summary of scripts/gpu_pmc_sq.sh passes.

    python scripts/pmc_sq_summary.py gpurun_out/pmcsq_1 gpurun_out/pmcsq_2 ...
    python scripts/pmc_sq_summary.py --json OUT.json CONFIG DIR1 DIR2 ...

With --json, the per-direction integer roofline of the dominant crypto
kernel is stored under CONFIG in OUT.json (bench.py attaches it as
roofline.int_frac / lds_frac):
  valu_frac = SQ_INSTS_VALU / (kernel time x 1024 SIMDs x R), R = 0.833 G
              wave-instructions/s per SIMD, the measured v_xor / v_bitop3
              issue rate at 4 waves/SIMD (profiles/r01_ubench_valu_rates.log:
              54.6 T lane-ops/s / 65536 lanes); 3-operand ops (v_add3,
              v_perm, v_alignbit) issue at ~0.6 of it, so 1.0 is not
              reachable by a mixed stream
  lds_frac  = SQ_LDS_IDX_ACTIVE / (GRBM_GUI_ACTIVE / 8 x 256 CUs): both
              counters are summed over the 8 XCDs

Prints, for every k_ctr_hmac / k_gcm kernel, the counters averaged over
its launches (summed over XCDs/SEs as rocprofv3 reports them) and the
derived rates: VALU instructions per wave-cycle, LDS-array utilisation
(SQ_LDS_IDX_ACTIVE / (GRBM_GUI_ACTIVE/8 x 256 CUs)), bank-conflict
share and the effective clock (GRBM_GUI_ACTIVE / 8 / kernel time).
SQ_WAVE_CYCLES / SQ_ACTIVE_* / SQ_WAIT_* count quad-cycles
(MI355X_MICROARCH.md, per-instruction constants).
"""
import csv
import json
import sys
from collections import defaultdict

CRYPTO = ("k_ctr_fast_any", "k_ctr_fast_mk", "k_ctr_hmac", "k_gcm")
VALU_RATE = 54.56e12 / 65536   # wave-instructions/s per SIMD (v_xor, 4 w/S)
SIMDS = 1024


def main():
    args = sys.argv[1:]
    out = cfg = None
    if args and args[0] == "--json":
        out, cfg, args = args[1], args[2], args[3:]
    acc = defaultdict(lambda: defaultdict(list))
    dur = defaultdict(list)
    res = {}
    for d in args:
        for r in csv.DictReader(open(d + "/run_counter_collection.csv")):
            k = r["Kernel_Name"]
            if not any(c in k for c in CRYPTO):
                continue
            v = float(r["Counter_Value"])
            acc[k][r["Counter_Name"]].append(v)
            if "End_Timestamp" in r and r.get("Start_Timestamp"):
                dur[k].append(int(r["End_Timestamp"]) -
                              int(r["Start_Timestamp"]))
    for k, cs in acc.items():
        m = {c: sum(v) / len(v) for c, v in cs.items() if max(v) > 0}
        if not m:
            continue
        print(k)
        for c in sorted(m):
            print("   %-24s %16.0f" % (c, m[c]))
        t = sorted(dur[k])[len(dur[k]) // 2] if dur[k] else 0
        if t and "GRBM_GUI_ACTIVE" in m:
            print("   clock_GHz                %16.3f" %
                  (m["GRBM_GUI_ACTIVE"] / 8 / t))
        if "SQ_INSTS_VALU" in m and "SQ_WAVE_CYCLES" in m:
            print("   valu_per_wave_quadcycle  %16.3f" %
                  (m["SQ_INSTS_VALU"] / m["SQ_WAVE_CYCLES"]))
        if "SQ_LDS_IDX_ACTIVE" in m and "GRBM_GUI_ACTIVE" in m:
            print("   lds_array_util           %16.3f" %
                  (m["SQ_LDS_IDX_ACTIVE"] / (m["GRBM_GUI_ACTIVE"] / 8 * 256)))
        if "SQ_LDS_BANK_CONFLICT" in m and "SQ_LDS_IDX_ACTIVE" in m:
            print("   bank_conflict_share      %16.3f" %
                  (m["SQ_LDS_BANK_CONFLICT"] / m["SQ_LDS_IDX_ACTIVE"]))
        e = {"kernel": k, "kernel_ns": t}
        if t and "SQ_INSTS_VALU" in m:
            e["valu_frac"] = m["SQ_INSTS_VALU"] / (t * 1e-9 * SIMDS *
                                                   VALU_RATE)
            print("   valu_frac                %16.3f" % e["valu_frac"])
        if "SQ_LDS_IDX_ACTIVE" in m and "GRBM_GUI_ACTIVE" in m:
            e["lds_frac"] = m["SQ_LDS_IDX_ACTIVE"] / (
                m["GRBM_GUI_ACTIVE"] / 8 * 256)
        if t and "GRBM_GUI_ACTIVE" in m:
            e["clock_GHz"] = m["GRBM_GUI_ACTIVE"] / 8 / t
        for c in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_WAVES"):
            if c in m:
                e[c] = m[c]
        args_ = [x.strip() for x in k[k.index("<") + 1:k.index(">")]
                 .split(",")] if "<" in k else []
        prot = args_[2] if ("k_ctr_hmac<" in k) else \
            (args_[1] if len(args_) > 1 else "?")
        dn = "protect" if prot == "true" else "unprotect"
        if t and (dn not in res or t > res[dn]["kernel_ns"]):
            res[dn] = e
    if out:
        try:
            allr = json.load(open(out))
        except (OSError, ValueError):
            allr = {}
        allr[cfg] = res
        json.dump(allr, open(out, "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
