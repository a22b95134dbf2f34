"""Multi-GPU batch resolution inside one process: the path shards, so a batch is
split into byte-balanced contiguous string ranges (ie_shard_bounds: binary search on the
offsets), the inserts table is built once and replicated device-to-device (ie_table_replicate:
hipMemcpyPeer, over xGMI between MI355X GPUs), and every shard is resolved on its own device and
stream concurrently (one host thread and one ie_exec per shard: ctypes releases the GIL in the
library calls). There is no collective: the results are concatenated in string order.

The benchmark's multi-GPU mode is one process per GPU instead (bench.py under
torch.distributed.run); this is the library form for a caller that owns several devices.
"""
import copy
import ctypes
from concurrent.futures import ThreadPoolExecutor

import numpy as np

from . import _native as N
from .interpolation_engine import InsertsTable


def shard_bounds(offsets, n_shards):
    """first[k] .. first[k+1] = the strings of shard k (n_shards + 1 entries)"""
    offs = np.ascontiguousarray(offsets, dtype=np.uint64)
    n = offs.size - 1
    first = np.zeros(n_shards + 1, np.uint64)
    N.check(N.lib().ie_shard_bounds(offs.ctypes.data, n, n_shards, first.ctypes.data), "ie_shard_bounds")
    return first


class MultiDevice:
    """One inserts dict resolved on several devices (a device may repeat: each entry is a shard
    with its own exec and table replica)."""

    def __init__(self, inserts, devices, dialect="py", clock=None, has_inserts_dir=False):
        self.devices = list(devices)
        if not self.devices:
            raise ValueError("no devices")
        self.tables = [InsertsTable(inserts, dialect=dialect, clock=clock, device=self.devices[0],
                                    has_inserts_dir=has_inserts_dir)]
        for d in self.devices[1:]:
            h = ctypes.c_void_p()
            N.check(N.lib().ie_table_replicate(self.tables[0].h, d, ctypes.byref(h)), "ie_table_replicate")
            rep = copy.copy(self.tables[0])
            rep.h, rep.device = h, d
            self.tables.append(rep)
        self.execs = [N.Exec(d) for d in self.devices]

    def close(self):
        for t in self.tables:
            t.close()
        self.tables = []

    def run(self, strings):
        """(status, payload) per string, as InsertsTable.run, the batch split over the devices"""
        strings = list(strings)
        _, offs = N.pack(strings)
        first = shard_bounds(offs, len(self.devices))

        def one(k):
            lo, hi = int(first[k]), int(first[k + 1])
            return self.tables[k].run(strings[lo:hi], exec_=self.execs[k]) if lo < hi else []
        with ThreadPoolExecutor(len(self.devices)) as pool:
            parts = list(pool.map(one, range(len(self.devices))))
        return [r for p in parts for r in p]
