"""Per-workgroup phases of a fused plan + crypto launch (RE_SRTP_FZ_TIMING
stamps, 8 u64 per workgroup in ticket order: start, ticket+T4 fill,
headers, look-back, done, blockIdx, XCC), wall clock at 100 MHz."""
import sys
import numpy as np

a = np.fromfile(sys.argv[1], dtype=np.uint64).reshape(-1, 8).astype(np.int64)
t0 = a[:, 0].min()
us = (a[:, :5] - t0) / 100.0          # 100 MHz -> us
ph = np.diff(us, axis=1)
print("workgroups %d, launch span %.1f us" % (len(a), us[:, 4].max()))
for k, nm in enumerate(("ticket+fill", "headers", "look-back", "crypto")):
    print("  %-12s mean %6.2f  p50 %6.2f  p90 %6.2f  max %6.2f us" % (
        nm, ph[:, k].mean(), np.median(ph[:, k]), np.percentile(ph[:, k], 90),
        ph[:, k].max()))
pre = ph[:, :3].sum(axis=1)
print("  plan total   mean %6.2f us; first 256 wg: %.2f, rest: %.2f" % (
    pre.mean(), pre[:256].mean(), pre[256:].mean()))
st = us[:, 0]
print("  start of ticket k (first 8 / at 256, 512, 768):",
      np.round(np.sort(st)[:8], 1), np.round(np.sort(st)[[256, 512, 768]], 1))
print("  blockIdx == ticket: %.3f; XCCs %s" % (
    (a[:, 5] == np.arange(len(a))).mean(), np.unique(a[:, 6])))
