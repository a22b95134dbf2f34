"""Diagnostic: config-4 sample through the device path vs the oracle; prints the mismatches."""
import ctypes, sys, os
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
import test_gpu_parity as T
from oracle import oracle as O
N = T.N
h, kvp, nkv = T._synth(4)
table = T._table_from_kv(kvp, nkv)
x = N.Exec(0)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 200_000
buf, offs = T._host_strings(h, 0, n)
d_bytes = N.DeviceBuffer.from_numpy(x, buf)
d_off = N.DeviceBuffer.from_numpy(x, offs)
r = T._device_run(x, table, d_bytes, d_off, n)
ref = O.Oracle.from_kv(ctypes.cast(kvp, ctypes.c_void_p), nkv, "py", clock=T.CLOCK)
oo = r.off.to_numpy(np.uint64, n + 1)
ob = r.bytes.to_numpy(np.uint8, r.total()).tobytes()
st = r.status.to_numpy(np.uint8, n)
bad = 0
kinds = {}
for i in range(n):
    s = buf[int(offs[i]):int(offs[i + 1])].tobytes()
    rs, rout, _ = ref.interpolate(s)
    g = ob[int(oo[i]):int(oo[i + 1])].decode("utf-8", "replace")
    if N.STATUS_NAMES[st[i]] != rs or (rs == "OK_STR" and g != rout):
        bad += 1
        k = ("esc" if b"\\{" in s else "") + ("cval" if b"{c-" in s else "") + ("miss" if b"{zz-" in s else "")
        kinds[k] = kinds.get(k, 0) + 1
        if bad <= 12:
            print(i, repr(s.decode()), "\n   gpu", N.STATUS_NAMES[st[i]], repr(g), "\n   ref", rs, repr(rout), flush=True)
print("mismatches", bad, "of", n, kinds)
