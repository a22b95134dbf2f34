"""Phase durations of a stamp dump (IE_DEBUG_STAMPS), chain-job kernel: slots 0 start, 1 staged,
8 parsed + job scan, 9 jobs written, 10 wave 0's jobs resolved, 11 all jobs resolved, 12 combined,
2 evaluated, 3 literal, 4 output built, 5 streamed out."""
import sys

import numpy as np

a = np.fromfile(sys.argv[1], dtype=np.uint64).reshape(-1, 16).astype(np.int64)
order = [(0, 1, "stage"), (1, 8, "parse+scan"), (8, 9, "job write"), (9, 10, "resolve(w0)"), (10, 11, "resolve barrier"),
         (11, 12, "combine"), (12, 2, "exact+status"), (2, 3, "literal"), (3, 4, "scan+build"), (4, 5, "lookback+stream")]
ok = np.all(a[:, [0, 1, 2, 3, 4, 5, 8, 9, 10, 11, 12]] > 0, axis=1)
print("tiles with every stamp: %d of %d" % (ok.sum(), len(a)))
b = a[ok]
for x, y, nm in order:
    d = (b[:, y] - b[:, x]) / 100.0
    print("%-16s mean %6.2f us  p10 %6.2f  p90 %6.2f" % (nm, d.mean(), *np.percentile(d, [10, 90])))
life = (b[:, 5] - b[:, 0]) / 100.0
print("life mean %.2f us; span %.3f ms" % (life.mean(), (b[:, 5].max() - b[:, 0].min()) / 1e5))
# inside wave 0's first resolve call: 6 round-0 keys hashed, 13 pilots arrived, 14 entries arrived, 15 round-1 entries
m = np.all(b[:, [6, 13, 14]] > 0, axis=1)
if m.any():
    c = b[m]
    print("round 0: keys %.2f us, pilot %.2f us, entry %.2f us" % (((c[:, 6] - c[:, 9]) / 100).mean(), ((c[:, 13] - c[:, 6]) / 100).mean(), ((c[:, 14] - c[:, 13]) / 100).mean()))
    m2 = c[:, 15] > 0
    if m2.any():
        print("round 1 (keys+pilot+entry) %.2f us; after -> resolved %.2f us" % (((c[m2, 15] - c[m2, 14]) / 100).mean(), ((c[m2, 10] - c[m2, 15]) / 100).mean()))
# the slowest tiles (a slow tile holds back every later tile's look-back)
print("life p50 %.2f p99 %.2f p99.9 %.2f max %.2f us" % (*np.percentile(life, [50, 99, 99.9]), life.max()))
idx = np.argsort(-life)[:8]
for t in idx:
    row = b[t]
    print("  tile %6d life %8.2f us: " % (np.flatnonzero(ok)[t], life[t]) +
          " ".join("%s %.1f" % (nm, (row[y] - row[x]) / 100.0) for x, y, nm in order))
