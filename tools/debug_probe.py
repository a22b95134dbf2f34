"""GPU diagnostic: device vs host lookup of every key of the golden tables (ie_debug_probe)."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as G  # noqa: E402
from tests.conftest import load_golden  # noqa: E402

G.build()
PKG = G.load_package()
N = PKG._native
lib = N.lib()
lib.ie_debug_probe.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint64)]
tables = load_golden("tables.json")
bad = 0
for ti, tab in enumerate(tables):
    t = PKG.InsertsTable(tab, dialect="py", clock=(12, 34, 56))
    for k in list(tab) + ["HH:MM", "HH:MM:SS", "missing-key"]:
        kb = k.encode("utf-8", "surrogatepass")
        out = (ctypes.c_uint64 * 16)()
        N.check(lib.ie_debug_probe(t.h, kb, len(kb), out), "probe")
        o = list(out)
        dev = (o[0] | (o[1] << 32), o[2], o[3])
        host = (o[7] | (o[8] << 32), o[9], o[10])
        fb = o[4] - (1 << 64) if o[4] >> 63 else o[4]
        fs = o[5] - (1 << 64) if o[5] >> 63 else o[5]
        where = o[11] - (1 << 64) if o[11] >> 63 else o[11]
        fw = o[12] - (1 << 64) if o[12] >> 63 else o[12]
        good = dev == host and fb == where and (fs == where or fs == -2) and fw == where and o[13] == (1 << 64) - 1 and (where < 0 or o[14] == o[15])
        if not good:
            bad += 1
            if bad < 30:
                print("t%d %r dev(h=%x s=%d,%d) host(h=%x s=%d,%d) fb=%d fs=%d fw=%d agree=%x off %d/%d at=%d mask=%d" %
                      (ti, k, dev[0], dev[1], dev[2], host[0], host[1], host[2], fb, fs, fw, o[13], o[14], o[15], where, o[6]))
print("bad", bad)
