#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes into the
per-launch HBM traffic of the crypto kernels (profiles/*_pmc_traffic.json).

MI355X_MICROARCH.md (HBM / rocprofv3): FETCH_SIZE and WRITE_SIZE are in
KiB, come from separate passes, and on gfx950 FETCH_SIZE reports half of
the bytes of a wide streaming read -- doubled here.
usage: pmc_summary.py OUT.json CONFIG_NAME gpurun_out/pmc_FETCH_SIZE gpurun_out/pmc_WRITE_SIZE
"""
import csv
import json
import sys

# the crypto kernels: k_ctr_fast_any / k_ctr_fast_mk (lean: device-planned
# single key / per-lane keys),
# k_ctr_hmac / k_ctr_hmac_any (general compact), k_gcmu / k_gcm
CRYPTO = ("k_ctr_fast_any", "k_ctr_fast_mk", "k_ctr_hmac", "k_gcm")


def per_kernel(path, counter):
    rows = list(csv.DictReader(open(path + "/run_counter_collection.csv")))
    agg = {}
    for r in rows:
        if r["Counter_Name"] != counter:
            continue
        name = r["Kernel_Name"]
        if not any(k in name for k in CRYPTO):
            continue
        v = float(r["Counter_Value"]) * 1024.0
        if v <= 0:
            continue          # class-guarded launches that exited at once
        agg.setdefault(name, []).append((int(r["Grid_Size"]), v))
    return agg


def main():
    out, cfg, fetch_dir, write_dir = sys.argv[1:5]
    f = per_kernel(fetch_dir, "FETCH_SIZE")
    w = per_kernel(write_dir, "WRITE_SIZE")
    res = {}
    try:
        res = json.load(open(out))
    except (OSError, ValueError):
        pass
    kern = {}
    for name in sorted(set(f) | set(w)):
        fv = [v for _, v in f.get(name, [])]
        wv = [v for _, v in w.get(name, [])]
        if not fv or not wv:
            continue
        args = [x.strip() for x in
                name[name.index("<") + 1:name.index(">")].split(",")]
        # k_ctr_hmac<NR, SHIFT, PROT, COMPACT, UNI>,
        # k_ctr_hmac_any<NR, PROT, UNI>, k_gcm<NR, PROT, ...>
        prot = args[2] if ("k_ctr_hmac" in name and
                           "k_ctr_hmac_any" not in name) else args[1]
        d = "protect" if prot == "true" else "unprotect"
        fb = 2.0 * sum(fv) / len(fv)
        wb = sum(wv) / len(wv)
        e = {"kernel": name, "fetch_bytes_x2": fb, "write_bytes": wb,
             "traffic_bytes_per_launch": fb + wb, "launches": len(fv),
             "grid": f[name][0][0]}
        if d not in kern or e["traffic_bytes_per_launch"] > \
                kern[d]["traffic_bytes_per_launch"]:
            kern[d] = e
    res[cfg] = kern
    json.dump(res, open(out, "w"), indent=1, sort_keys=True)
    print(json.dumps(res[cfg], indent=1))


if __name__ == "__main__":
    main()
