#!/usr/bin/env python3
"""Round-5 per-kernel PMC summary (profiles/r05_pmc.json): scripts/
pmc_r03.py's traffic and VALU / LDS issue floors, plus the co-issue
corrected issue-time estimate the bench reports.  The
estimate is not a hard floor: the GCM kernels run up to ~4 % under it.

    python scripts/pmc_r05.py OUT.json WORKLOAD FETCH_DIR WRITE_DIR SQ_DIR

A kernel's VALU and LDS instructions do not co-issue freely on gfx950
(profiles/r04_ubench_coissue.txt: a mixed body costs its larger half plus
c x its smaller half).  issue_floor_frac = max(V, L) + c x min(V, L), V and
L the VALU and LDS floors as fractions of the launch, c interpolated from
the measured rows at the kernel's waves/SIMD by its instruction forms:
the half-rate share of its VALU and the b128 share of its LDS time, at the
kernel's LDS:VALU ratio (1:3 rows for b32).  issue_sum_frac = V + L (the
round-4 'issue_frac').  The fused plan + crypto kernel (k_ctr_fused) runs
the lean kernel's per-packet body: its steady-chunk mix is k_ctr_fast_any's.
"""
import json
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import pmc_r03 as R  # noqa: E402

ROOT = R.ROOT
R.CRYPTO = R.CRYPTO + ("k_ctr_fused",)
WAVES = {"k_ctr_fast_mk": 3}        # 768-thread blocks; the rest 1024 (4)


def coissue_rows(path):
    """{waves: {(lds form, valu class, ratio tag): c}}"""
    rows = {}
    for ln in open(path):
        m = re.match(r"waves/SIMD=(\d+) (\d+) (b32|b128) \+ (\d+) (full|half)"
                     r"(?: \((1:\d)\))?.*\(mixed-max\)/\(sum-max\) ([\d.]+)",
                     ln)
        if m:
            w, _, form, _, cls, ratio, c = m.groups()
            rows.setdefault(int(w), {})[(form, cls, ratio)] = float(c)
    return rows


def coissue_c(rows, waves, cl):
    """c for a kernel with ISA classes cl (isa_mix 'classes')"""
    # rows measured at 4 and 8 waves/SIMD; the 3-wave multi-key kernel
    # takes the nearest (4)
    r = rows[8] if waves >= 8 else rows[4]
    nv = cl.get("fast", 0) + cl.get("slow", 0)
    h = cl.get("slow", 0) / nv if nv else 0.0
    b32 = (1 - h) * r[("b32", "full", "1:3")] + h * r[("b32", "half", "1:3")]
    b128 = (1 - h) * r[("b128", "full", None)] + h * r[("b128", "half", None)]
    lt = cl.get("lds", 0) + 4 * cl.get("lds_b128", 0)
    q = 4 * cl.get("lds_b128", 0) / lt if lt else 0.0
    return (1 - q) * b32 + q * b128


def main():
    out = sys.argv[1]
    argv = list(sys.argv)
    R.main()                            # writes OUT with the r03 fields
    res = json.load(open(out))
    mix = json.load(open(os.path.join(ROOT, "profiles", "r03_isa_mix.json")))
    rows = coissue_rows(os.path.join(ROOT, "profiles",
                                     "r04_ubench_coissue.txt"))
    for e in res["entries"]:
        if e["workload"] != argv[2]:
            continue
        name = e["kernel"].replace("k_ctr_fused", "k_ctr_fast_any")
        if name not in mix or "lds_floor_frac" not in e:
            continue
        base = e["kernel"].split("<")[0]
        c = coissue_c(rows, WAVES.get(base, 4), mix[name]["classes"])
        v, l = e["int_frac"], e["lds_floor_frac"]
        e["issue_sum_frac"] = v + l
        e["coissue_c"] = round(c, 4)
        e["issue_floor_frac"] = max(v, l) + c * min(v, l)
        e["issue_frac"] = e["issue_floor_frac"]
    json.dump(res, open(out, "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
