"""GPU diagnostic: find the strings of a golden table whose presence breaks a batch.
Runs every string alone, then tile-sized chunks, and prints mismatch indices (raw bytes)."""
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
TI = int(sys.argv[1]) if len(sys.argv) > 1 else 3
tables, interp = load_golden("tables.json"), load_golden("interp_py.jsonl")
strings = [r["s"] for r in interp if r["t"] == TI]
t = PKG.InsertsTable(tables[TI], dialect="py", clock=CLOCK)
ref = O.Oracle(tables[TI], "py", clock=CLOCK)
x = PKG.interpolation_engine.get_exec(0)


def run(ss):
    blob, offs = N.pack(ss)
    res = ctypes.POINTER(N.BatchRes)()
    bp = ctypes.c_char_p(blob)
    N.check(N.lib().ie_interpolate_batch(x.h, t.h, ctypes.cast(bp, ctypes.c_void_p), offs.ctypes.data,
                                         len(ss), ctypes.byref(res)), "batch")
    return N.batch_to_python(res)


def bad_of(ss, base=0):
    outs, sts, _ = run(ss)
    bad = []
    for k, (s, o, st) in enumerate(zip(ss, outs, sts)):
        rst, rout, _ = ref.interpolate(s)
        exp = rout.encode("utf-8", "surrogatepass") if rst == "OK_STR" else None
        if N.STATUS_NAMES[st] != rst or (rst == "OK_STR" and bytes(o) != exp):
            bad.append((base + k, s, N.STATUS_NAMES[st], bytes(o), rst, exp))
    return bad


alone = []
if os.environ.get("SKIP_ALONE"): strings_alone = []
else: strings_alone = strings
for k, s in enumerate(strings_alone):
    alone += bad_of([s], k)
print("alone: %d bad" % len(alone))
for b in alone[:20]:
    print("  ", b)
for c0 in range(0, len(strings), 256):
    bad = bad_of(strings[c0:c0 + 256], c0)
    print("chunk %d: %d bad, idx %s" % (c0, len(bad), [b[0] for b in bad][:40]))
whole = bad_of(strings)
print("whole: %d bad, idx range %s" % (len(whole), (whole[0][0], whole[-1][0]) if whole else None))


def fails(ss):
    return len(bad_of(ss)) > 0


# greedy linear minimisation of the failing chunk: drop each string if the rest still fails
S = strings[768:]
print("chunk fails:", fails(S), flush=True)
k = 0
while k < len(S):
    T2 = S[:k] + S[k + 1:]
    if T2 and fails(T2):
        S = T2
    else:
        k += 1
print("minimal failing set (%d):" % len(S))
for s in S:
    print("   %r" % s)
outs, sts, vids = run(S)
for s, o, st in zip(S, outs, sts):
    print("   got %s %r  exp %r" % (N.STATUS_NAMES[st], bytes(o), ref.interpolate(s)))
