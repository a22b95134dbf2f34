"""Summarise a per-tile phase-stamp dump (IE_DEBUG_STAMPS): phase durations, concurrency."""
import sys

import numpy as np

a = np.fromfile(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/stamps.bin", dtype=np.uint64).reshape(-1, 16)
t = a[:, :6].astype(np.int64)
ph = np.diff(t, axis=1) / 100.0
for k, nm in enumerate(["stage+classify", "eval", "literal", "scan+lookback", "emit"]):
    x = ph[:, k]
    print("%-15s mean %8.2f us  p50 %8.2f  p99 %8.2f  max %8.2f" % (nm, x.mean(), np.median(x), np.percentile(x, 99), x.max()))
life = (t[:, 5] - t[:, 0]) / 100.0
ev = np.concatenate([np.stack([t[:, 0], np.ones(len(t))], 1), np.stack([t[:, 5], -np.ones(len(t))], 1)])
ev = ev[np.argsort(ev[:, 0], kind="stable")]
print("tiles %d  life mean %.1f us  span %.1f us  max concurrent %d" % (len(t), life.mean(), (t[:, 5].max() - t[:, 0].min()) / 100, np.cumsum(ev[:, 1]).max()))
