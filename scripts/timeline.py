"""Print the last N kernels of a rocprofv3 kernel trace with gaps (us)."""
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
sel = rows[-int(sys.argv[2] if len(sys.argv) > 2 else 40):]
t0 = int(sel[0]['Start_Timestamp'])
prev = None
for r in sel:
    s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
    gap = (s - prev) / 1000 if prev else 0
    print(f"{(s - t0) / 1000:9.1f} gap{gap:7.1f} dur{(e - s) / 1000:8.1f} "
          f"{r['Kernel_Name'][:60]}")
    prev = e
