"""Per-step GPU time split of a bench.py kernel trace (rocprofv3
--kernel-trace csv): steps start at each protect crypto launch (NAME,
default the first kernel whose name contains 'k_ctr_fast_any<10, true>' or
'k_ctr_fused'); prints, per step, wall span, crypto kernels, other kernels
and idle gaps (us), then the mean over the last K steps."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
K = int(sys.argv[2]) if len(sys.argv) > 2 else 20
rows.sort(key=lambda r: int(r['Start_Timestamp']))
CRYPTO = ('k_ctr_fast_any', 'k_ctr_fused', 'k_gcmu', 'k_ctr_fast_mk',
          'k_ctr_fast_rtcp')


def is_start(name):
    return ('k_ctr_fast_any<10, true>' in name or
            'k_ctr_fused<10, true>' in name or 'k_gcmu<14, true>' in name or
            'k_ctr_fast_rtcp<10, true>' in name or
            'k_ctr_fast_mk<10, true>' in name)


starts = [k for k, r in enumerate(rows) if is_start(r['Kernel_Name'])]
# a step begins at the first kernel after the previous step's last crypto
# launch: walk back from each protect launch over its planner kernels
steps = []
for a, b in zip(starts[:-1], starts[1:]):
    steps.append((a, b))
steps = steps[-K:]
tot = {"span": 0.0, "crypto": 0.0, "other": 0.0, "gap": 0.0}
other_names = {}
for a, b in steps:
    t0 = int(rows[a]['Start_Timestamp'])
    t1 = int(rows[b]['Start_Timestamp'])
    cr = ot = busy_end = 0
    prev_end = t0
    gap = 0
    for r in rows[a:b]:
        s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
        if s > prev_end:
            gap += s - prev_end
        prev_end = max(prev_end, e)
        d = e - s
        if any(c in r['Kernel_Name'] for c in CRYPTO):
            cr += d
        else:
            ot += d
            nm = r['Kernel_Name'].split('(')[0][:48]
            other_names[nm] = other_names.get(nm, 0) + d
    gap += max(0, t1 - prev_end)
    for k, v in (("span", t1 - t0), ("crypto", cr), ("other", ot),
                 ("gap", gap)):
        tot[k] += v / 1000.0
n = len(steps)
print("steps %d: span %.1f us, crypto %.1f, other kernels %.1f, idle %.1f"
      % (n, tot["span"] / n, tot["crypto"] / n, tot["other"] / n,
         tot["gap"] / n))
for nm, v in sorted(other_names.items(), key=lambda x: -x[1]):
    print("  %-48s %7.1f us/step" % (nm, v / 1000.0 / n))
