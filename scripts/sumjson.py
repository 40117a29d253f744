#!/usr/bin/env python3
"""One summary line per bench.py JSON line in the given files:
value, Mpkt/s, ms/step, round-trip check and the two heaviest kernels."""
import json
import sys

for path in sys.argv[1:]:
    try:
        lines = open(path).read().strip().splitlines()
    except OSError as e:
        print(path, "missing:", e)
        continue
    for l in lines:
        if not l.startswith("{"):
            continue
        d = json.loads(l)
        ks = (d.get("roofline") or {}).get("kernels", [])[:2]
        print(path.split("/")[-1], d["value"], d.get("mpkt_s"),
              d["ms_per_step"], d.get("verified_roundtrip"),
              [(k["dir"], k["avg_ms"]) for k in ks])
