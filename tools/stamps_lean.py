"""Phase durations of a k_lean stamp dump (IE_DEBUG_STAMPS): per 256-string tile a row of 16 words,
four per wave: 0 start, 1 resolved (stage + parse + lookups), 2 claimed (the tile's claim barrier
passed), 3 stored."""
import sys

import numpy as np

a = np.fromfile(sys.argv[1], dtype=np.uint64).reshape(-1, 16).astype(np.int64)
w = a.reshape(-1, 4, 4).reshape(-1, 4)  # one row per wave-tile
w = w[(w[:, 0] > 0) & (w[:, 3] > 0)]
names = ["start", "resolved", "claimed", "stored"]
print("wave-tiles %d" % len(w))
for x in range(3):
    d = (w[:, x + 1] - w[:, x]) / 100.0
    print("%-9s -> %-9s mean %6.2f us  p10 %6.2f  p90 %6.2f" % (names[x], names[x + 1], d.mean(), *np.percentile(d, [10, 90])))
life = (w[:, 3] - w[:, 0]) / 100.0
span = (w[:, 3].max() - w[:, 0].min()) / 1e5
print("life mean %.2f us p50 %.2f p99 %.2f; span %.3f ms; wave-tiles in flight %.0f"
      % (life.mean(), *np.percentile(life, [50, 99]), span, life.sum() / (span * 1e3)))
