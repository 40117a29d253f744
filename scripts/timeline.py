"""Print kernels of a rocprofv3 kernel trace with gaps (us): the last N, or
(--crypto) the N up to and including the last crypto launch (the timed
region of a bench run, not the verification kernels after it)."""
import csv
import sys

CRYPTO = ('k_ctr_fast_any', 'k_ctr_fused', 'k_gcmu', 'k_ctr_fast_mk',
          'k_ctr_fast_rtcp')
args = [a for a in sys.argv[1:] if not a.startswith('--')]
rows = list(csv.DictReader(open(args[0])))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
N = int(args[1]) if len(args) > 1 else 40
end = len(rows)
if '--crypto' in sys.argv:
    last = [k for k, r in enumerate(rows)
            if any(c in r['Kernel_Name'] for c in CRYPTO)]
    if last:
        end = last[-1] + 3
sel = rows[max(0, end - N):end]
t0 = int(sel[0]['Start_Timestamp'])
prev = None
for r in sel:
    s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
    gap = (s - prev) / 1000 if prev else 0
    print(f"{(s - t0) / 1000:9.1f} gap{gap:7.1f} dur{(e - s) / 1000:8.1f} "
          f"{r['Kernel_Name'][:60]}")
    prev = e
