"""GPU diagnostic: run a few strings of one golden table singly and print raw results."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as G  # noqa: E402
from oracle import oracle as O  # noqa: E402
from tests.conftest import load_golden  # noqa: E402

G.build()
PKG = G.load_package()
N = PKG._native
TI = int(sys.argv[1])
cases = [c.encode().decode("unicode_escape").encode("latin-1").decode("utf-8") for c in sys.argv[2:]]
tab = load_golden("tables.json")[TI]
t = PKG.InsertsTable(tab, dialect="py", clock=(12, 34, 56))
ref = O.Oracle(tab, "py", clock=(12, 34, 56))
x = PKG.interpolation_engine.get_exec(0)
N.lib().ie_exec_set_timing(x.h, 1)
for s in cases:
    blob, offs = N.pack([s])
    res = ctypes.POINTER(N.BatchRes)()
    bp = ctypes.c_char_p(blob)
    N.check(N.lib().ie_interpolate_batch(x.h, t.h, ctypes.cast(bp, ctypes.c_void_p), offs.ctypes.data, 1,
                                         ctypes.byref(res)), "batch")
    outs, sts, vids = N.batch_to_python(res)
    tm = N.Timing()
    N.lib().ie_exec_timing(x.h, ctypes.byref(tm))
    print(repr(s), "->", N.STATUS_NAMES[sts[0]], bytes(outs[0]), "| literal", tm.n_complex, "| exp", ref.interpolate(s))
