"""Phase durations of a stamp dump (IE_DEBUG_STAMPS) by tile-index bucket, and look-back waits
against the predecessor's publication time."""
import sys

import numpy as np

a = np.fromfile(sys.argv[1], dtype=np.uint64).reshape(-1, 16)
t = a[:, :6].astype(np.int64)
t0 = t[:, 0].min()
ph = np.diff(t, axis=1) / 100.0
n = len(t)
names = ["stage", "eval", "lit", "lookb", "emit"]
for lo in range(0, n, n // 8):
    sl = slice(lo, min(n, lo + n // 8))
    print("tiles %6d-%6d start %7.1f us " % (lo, sl.stop, (t[sl, 0].min() - t0) / 100) +
          " ".join("%s %6.2f" % (nm, ph[sl, k].mean()) for k, nm in enumerate(names)))
# how many tiles are in each phase over time (steady state)
T = np.arange(t[:, 0].min(), t[:, 5].max(), 1000)
mid = T[len(T) // 2]
inph = [(np.sum((t[:, k] <= mid) & (t[:, k + 1] > mid))) for k in range(5)]
print("at t=%.0f us: tiles per phase" % ((mid - t0) / 100), dict(zip(names, inph)))
# publication of the aggregate = end of 'lit' (t[:,3]); inclusive = end of lookback (t[:,4])
incl = t[:, 4]
lag = (t[1:, 3] - incl[:-1]) / 100.0  # tile i reaches look-back minus tile i-1's inclusive time
print("tile reaches lookback relative to predecessor's inclusive: p10 %.2f p50 %.2f p90 %.2f us" % tuple(np.percentile(lag, [10, 50, 90])))
order = np.argsort(t[:, 0])
print("start order == tile order fraction: %.3f" % np.mean(np.diff(t[order, 0]) >= 0))
life = (t[:, 5] - t[:, 0]) / 100
print("life p10 %.1f p50 %.1f p90 %.1f p99 %.1f" % tuple(np.percentile(life, [10, 50, 90, 99])))
xcc = (a[:, 7] >> 32).astype(np.int64)
for x in range(8):
    m = xcc == x
    if m.any():
        print("xcc %d tiles %5d life %.1f stage %.2f eval %.2f lookb %.2f emit %.2f" % (x, m.sum(), life[m].mean(), ph[m, 0].mean(), ph[m, 1].mean(), ph[m, 3].mean(), ph[m, 4].mean()))
# slot 6: end of the chain evaluator's parse (wave 0), when written
p6 = a[:, 6].astype(np.int64)
ok = (p6 > t[:, 1]) & (p6 < t[:, 2])
if ok.any():
    print("eval: parse %.2f us, rounds+exact %.2f us (tiles with the stamp: %d)" % (((p6 - t[:, 1])[ok] / 100).mean(), ((t[:, 2] - p6)[ok] / 100).mean(), ok.sum()))
# slots 8..13: round r pilots arrived (8 + 2r), entries arrived (9 + 2r)
r0 = a[:, 8].astype(np.int64)
if (r0 > 0).any():
    prev = p6
    for r in range(3):
        pa, ea = a[:, 8 + 2 * r].astype(np.int64), a[:, 9 + 2 * r].astype(np.int64)
        m = (pa > 0) & (ea > 0) & (prev > 0)
        if not m.any():
            break
        print("round %d: keys+pilot %.2f us, entries %.2f us (tiles %d)" % (r, ((pa - prev)[m] / 100).mean(), ((ea - pa)[m] / 100).mean(), m.sum()))
        prev = ea
    m = prev > 0
    print("after last round -> eval end %.2f us" % (((t[:, 2] - prev)[m]) / 100).mean())
