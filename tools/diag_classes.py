"""Diagnostic: k_resolve time per string class of config 4 (each class replicated to 2M strings)."""
import ctypes, sys, os, re
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
import test_gpu_parity as T
N = T.N
h, kvp, nkv = T._synth(4)
table = T._table_from_kv(kvp, nkv)
x = N.Exec(0)
n = 400_000
buf, offs = T._host_strings(h, 0, n)
b = buf.tobytes()
ss = [b[int(offs[i]):int(offs[i + 1])] for i in range(n)]
def depth(s):
    d = m = 0
    for c in s:
        if c == 0x7B: d += 1; m = max(m, d)
        elif c == 0x7D: d -= 1
    return m
classes = {
    "plain_d12": [s for s in ss if depth(s) <= 2 and b"\\" not in s and b"{c-" not in s and b"{zz-" not in s],
    "d3": [s for s in ss if depth(s) == 3 and b"\\" not in s and b"{c-" not in s and b"{zz-" not in s],
    "d4": [s for s in ss if depth(s) == 4 and b"\\" not in s and b"{c-" not in s and b"{zz-" not in s],
    "esc": [s for s in ss if b"\\" in s and b"{c-" not in s and b"{zz-" not in s],
    "cval": [s for s in ss if b"{c-" in s],
    "miss": [s for s in ss if b"{zz-" in s],
    "all": ss,
}
M = 2_000_000
for name, lst in classes.items():
    rep = (lst * (M // max(1, len(lst)) + 1))[:M]
    lens = np.array([len(s) for s in rep], np.uint64)
    o = np.zeros(M + 1, np.uint64); o[1:] = np.cumsum(lens)
    bb = np.frombuffer(b"".join(rep) + b"\0" * 16, np.uint8)
    d_b = N.DeviceBuffer.from_numpy(x, bb); d_o = N.DeviceBuffer.from_numpy(x, o)
    r = T._device_run(x, table, d_b, d_o, M)
    x.set_timing(True)
    N.check(N.lib().ie_interpolate_device(x.h, table, d_b.ptr, d_o.ptr, M, ctypes.byref(r.out)), "run")
    tm = x.timing(); x.set_timing(False)
    print("%-10s %6d distinct  %8.3f ms for %d strings  lit=%d exact=%d" % (name, len(lst), tm.resolve_ms, M,
          tm.n_complex, tm.n_exact), flush=True)
