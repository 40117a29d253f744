"""one line per bench JSON file: value, step time, dominant kernel, folds"""
import json
import sys

for f in sys.argv[1:]:
    try:
        d = json.loads(open(f).read().strip().splitlines()[-1])
    except Exception as e:  # noqa: BLE001 -- a failed run's file
        print(f"{f:40s} ERR {e}")
        continue
    r = d.get("roofline") or {}
    print(f"{f:40s} {d.get('value')} {d.get('unit')} ms={d.get('ms_per_step')}"
          f" {r.get('kernel')} {r.get('avg_launch_ms')} frac={r.get('frac')}"
          f" folds={d.get('folds')} plans={d.get('plans')}")
