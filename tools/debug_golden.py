"""GPU diagnostic: run the golden vectors through the C ABI and print every mismatch with raw
output bytes (no decoding), plus the oracle's expectation."""
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
CLOCK = (12, 34, 56)
tables, interp = load_golden("tables.json"), load_golden("interp_py.jsonl")
by_table = {}
for row in interp:
    by_table.setdefault(row["t"], []).append(row)
nbad = 0
for ti, rows in sorted(by_table.items()):
    t = PKG.InsertsTable(tables[ti], dialect="py", clock=CLOCK)
    strings = [r["s"] for r in rows]
    blob, offs = N.pack(strings)
    x = PKG.interpolation_engine.get_exec(0)
    res = ctypes.POINTER(N.BatchRes)()
    bp = ctypes.c_char_p(blob)
    N.check(N.lib().ie_interpolate_batch(x.h, t.h, ctypes.cast(bp, ctypes.c_void_p), offs.ctypes.data,
                                         len(strings), ctypes.byref(res)), "batch")
    outs, sts, vids = N.batch_to_python(res)
    ref = O.Oracle(tables[ti], "py", clock=CLOCK)
    for s, o, st in zip(strings, outs, sts):
        rst, rout, rvid = ref.interpolate(s)
        name = N.STATUS_NAMES[st]
        exp = rout.encode("utf-8", "surrogatepass") if rst == "OK_STR" else None
        if name != rst or (rst == "OK_STR" and bytes(o) != exp):
            nbad += 1
            if nbad <= 40:
                print("t%d %r\n   got %s %r\n   exp %s %r" % (ti, s, name, bytes(o), rst, exp))
print("mismatches:", nbad, "of", len(interp))
