"""PCIe-inclusive rate of the host-buffer entry (ie_interpolate_batch: H2D, k_resolve, D2H) on a
config-3 sample; the device-resident rate is bench.py's `value`. Prints one JSON line."""
import ctypes, json, os, sys, time
import numpy as np
ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)
import __graft_entry__ as G

G.build()
N = G.load_package()._native
L = N.lib()
n = int(sys.argv[1]) if len(sys.argv) > 1 else 4_000_000
h = ctypes.c_void_p()
N.check(L.ie_synth_create(3, 0, ctypes.byref(h)), "synth")
kvp = ctypes.POINTER(N.KV)()
nkv = L.ie_synth_kv(h, ctypes.byref(kvp))
x = N.Exec(0)
t = ctypes.c_void_p()
clk = N.Clock(12, 34, 56)
N.check(L.ie_table_build(ctypes.cast(kvp, ctypes.c_void_p), nkv, 0, ctypes.byref(clk), 0, 0, ctypes.byref(t)), "table")
offs = np.zeros(n + 1, np.uint64)
tot = ctypes.c_uint64()
N.check(L.ie_synth_strings_host(h, 0, n, None, 0, offs.ctypes.data, ctypes.byref(tot)), "len")
buf = np.zeros(int(tot.value) + 16, np.uint8)
N.check(L.ie_synth_strings_host(h, 0, n, buf.ctypes.data, buf.size, offs.ctypes.data, ctypes.byref(tot)), "fill")
times = []
for k in range(4):
    b = ctypes.POINTER(N.BatchRes)()
    t0 = time.perf_counter()
    N.check(L.ie_interpolate_batch(x.h, t, buf.ctypes.data, offs.ctypes.data, n, ctypes.byref(b)), "batch")
    times.append(time.perf_counter() - t0)
    L.ie_batch_free(b)
best = min(times[1:])
print(json.dumps({"what": "ie_interpolate_batch (pageable host buffers: H2D + k_resolve + D2H + status scan)",
                  "strings": n, "input_bytes": int(tot.value), "s_per_call": round(best, 4),
                  "input_MB_per_s": round(int(tot.value) / best / 1e6, 1)}))
