"""Summarise gpurun_out/ab_*.json (scripts/gpu_ab.sh): value, step time
and the per-direction crypto kernel times of each run."""
import glob, json, sys
for f in sorted(glob.glob((sys.argv[1] if len(sys.argv) > 1 else "gpurun_out")
                          + "/ab_*.json")):
    try:
        d = json.loads(open(f).read().strip().splitlines()[-1])
    except Exception as e:      # a failed run: show why
        print(f, "unreadable:", e)
        continue
    big = [k for k in d["roofline"]["kernels"] if k["avg_ms"] > 0.1]
    print(f.split("/")[-1], d["value"], d["ms_per_step"],
          sorted((k["dir"], round(k["avg_ms"], 4)) for k in big))
