"""Phase durations of a stamp dump (IE_DEBUG_STAMPS) with whatever stamps the run wrote: slots
0 start, 1 staged, 8 parsed + job scan, 9 jobs written, 10 wave 0's jobs resolved, 11 all jobs
resolved, 12 combined, 2 evaluated, 3 literal, 4 output built, 5 written out."""
import sys

import numpy as np

a = np.fromfile(sys.argv[1], dtype=np.uint64).reshape(-1, 16).astype(np.int64)
a = a[(a[:, 0] > 0) & (a[:, 5] > 0)]
chain = [0, 1, 8, 9, 10, 11, 12, 2, 3, 4, 5]
names = {0: "start", 1: "staged", 8: "parsed", 9: "jobs written", 10: "w0 resolved", 11: "resolved", 12: "combined",
         2: "evaluated", 3: "literal", 4: "built", 5: "written"}
have = [k for k in chain if np.all(a[:, k] > 0)]
print("tiles %d; stamps %s" % (len(a), have))
for x, y in zip(have, have[1:]):
    d = (a[:, y] - a[:, x]) / 100.0
    print("%-14s -> %-14s mean %6.2f us  p10 %6.2f  p90 %6.2f" % (names[x], names[y], d.mean(), *np.percentile(d, [10, 90])))
life = (a[:, 5] - a[:, 0]) / 100.0
span = (a[:, 5].max() - a[:, 0].min()) / 1e5
print("life mean %.2f us p50 %.2f p99 %.2f; span %.3f ms; tiles in flight (life x tiles / span) %.0f"
      % (life.mean(), *np.percentile(life, [50, 99]), span, life.sum() / (span * 1e3)))
