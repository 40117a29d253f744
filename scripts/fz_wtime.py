"""Per-wave end times of the fused plan + crypto kernel (diagnostic).

Build: NOMAP=1 scripts/build_variants.sh wtime -DFZ_WTIME
Run:   RE_SRTP_LIB=$PWD/re_amd/lib/variants/wtime.so python scripts/fz_wtime.py
bench.py's default config-2 step (protect then unprotect) runs once; the
stamps left are the unprotect launch's: per ticket its start, CU id and
each of the 16 waves' end (s_memrealtime, 100 MHz).  Prints how the
waves of a workgroup finish (the spread between the first and the last),
how many workgroups run over time and how long each CU is idle between
its workgroups."""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.argv = ["bench.py", "--steps", "1", "--warmup", "1", "--no-cpu-baseline"]
import bench  # noqa: E402

bench.main()
lib = ctypes.CDLL(os.environ["RE_SRTP_LIB"])
n = 1024
buf = np.zeros(24 * n, dtype=np.uint64)
assert lib.sgpu_fz_wtime(buf.ctypes.data_as(ctypes.c_void_p),
                         ctypes.c_size_t(buf.size)) == 0
a = buf.reshape(n, 24).astype(np.int64)
t0 = a[:, 0].min()
st = (a[:, 0] - t0) / 100.0
we = (a[:, 2:18] - t0) / 100.0
end = we.max(axis=1)
first = we.min(axis=1)
life = end - st
print("workgroups %d, span %.1f us, lifetime mean %.1f p50 %.1f" %
      (n, end.max(), life.mean(), np.median(life)))
print("first wave done at %.1f%% of the lifetime (mean), last-first spread "
      "mean %.1f us" % (100 * ((first - st) / life).mean(),
                        (end - first).mean()))
order = np.sort(we - st[:, None], axis=1) / life[:, None]
print("k-th wave to finish, fraction of lifetime:",
      " ".join("%.2f" % x for x in order.mean(axis=0)))
hw = a[:, 1]
cu = ((hw >> 8) & 0xF) | (((hw >> 13) & 0x7) << 4) | (((hw >> 16) & 0x3) << 7)
# CU idle between consecutive workgroups on the same hardware slot
gaps = []
for c in np.unique(cu):
    m = np.where(cu == c)[0]
    o = m[np.argsort(st[m])]
    gaps += list(st[o[1:]] - end[o[:-1]])
gaps = np.array(gaps)
print("hardware CU ids %d; gap between a CU's workgroups: mean %.2f p50 %.2f "
      "max %.2f us (%d gaps)" % (len(np.unique(cu)), gaps.mean(),
                                 np.median(gaps), gaps.max(), len(gaps)))
# the plan's barriers (thread 0): 0 ticket, 4 after the image fill, 1 the
# header writes, 2 the checks' ballot, 3 the look-back
pb = (a[:, [18, 22, 19, 20, 21]] - t0) / 100.0
names = ("ticket", "image fill", "headers", "checks", "look-back")
prev = st
for k, nm in enumerate(names):
    d = pb[:, k] - prev
    print("  plan %-10s mean %6.2f p50 %6.2f p90 %6.2f us" % (
        nm, d.mean(), np.median(d), np.percentile(d, 90)))
    prev = pb[:, k]
for t in np.linspace(0, end.max(), 11):
    print("  %7.1f us: running %4d" % (t, ((st <= t) & (end > t)).sum()))
