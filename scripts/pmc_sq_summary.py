#!/usr/bin/env python3
"""Per-kernel SQ counter summary of scripts/gpu_pmc_sq.sh passes.

    python scripts/pmc_sq_summary.py gpurun_out/pmcsq_1 gpurun_out/pmcsq_2 ...

Prints, for every k_ctr_hmac / k_gcm kernel, the counters averaged over
its launches (summed over XCDs/SEs as rocprofv3 reports them) and the
derived rates: VALU instructions per wave-cycle, LDS-array utilisation
(SQ_LDS_IDX_ACTIVE / (GRBM_GUI_ACTIVE/8 x 32 CUs-per-XCD)), bank-conflict
share and the effective clock (GRBM_GUI_ACTIVE / 8 / kernel time).
SQ_WAVE_CYCLES / SQ_ACTIVE_* / SQ_WAIT_* count quad-cycles
(MI355X_MICROARCH.md, per-instruction constants).
"""
import csv
import sys
from collections import defaultdict


def main():
    acc = defaultdict(lambda: defaultdict(list))
    dur = defaultdict(list)
    for d in sys.argv[1:]:
        for r in csv.DictReader(open(d + "/run_counter_collection.csv")):
            k = r["Kernel_Name"]
            if "k_ctr_hmac" not in k and "k_gcm" not in k:
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
                  (m["SQ_LDS_IDX_ACTIVE"] / (m["GRBM_GUI_ACTIVE"] / 8 * 32)))
        if "SQ_LDS_BANK_CONFLICT" in m and "SQ_LDS_IDX_ACTIVE" in m:
            print("   bank_conflict_share      %16.3f" %
                  (m["SQ_LDS_BANK_CONFLICT"] / m["SQ_LDS_IDX_ACTIVE"]))


if __name__ == "__main__":
    main()
