"""Diagnostic (not product): where a scalar interpolate_inserts call's time goes (tools/mirror_latency.py's
scalar case), layer by layer: the whole call, table_for, results, run, the raw ctypes call with and
without the result conversion; and after a one-key mutation, table_for (the in-place refresh) alone."""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def per_call(fn, n=3000):
    for _ in range(50):
        fn()
    best = 1e9
    for _ in range(5):
        t0 = time.perf_counter()
        for _ in range(n // 5):
            fn()
        best = min(best, (time.perf_counter() - t0) / (n // 5))
    return round(1e6 * best, 2)


def main():
    import __graft_entry__ as G
    G.check_built()
    pkg = G.load_package()
    ie = pkg.interpolation_engine
    N = pkg._native
    ins = ie.VersionedInserts({"k%d" % i: "v%d" % i for i in range(100)})
    ins["name"] = "Tom"
    ins["kv1"] = "nested"
    s = "Hello {name}, item {k7} and {k{k1}}"
    t = ie.table_for(ins)
    x = ie.get_exec(t.device)
    b = N.enc(s)
    offs1 = (ctypes.c_uint64 * 2)(0, len(b))
    res = ctypes.POINTER(N.BatchRes)()
    f = N.lib().ie_interpolate_batch

    def raw():
        f(x.h, t.h, b, offs1, 1, ctypes.byref(res))

    def raw_conv():
        f(x.h, t.h, b, offs1, 1, ctypes.byref(res))
        return N.batch_to_python(res)

    out = {"call": per_call(lambda: ie.interpolate_inserts(ins, s)),
           "table_for": per_call(lambda: ie.table_for(ins)),
           "results": per_call(lambda: t.results([s])),
           "run": per_call(lambda: t.run([s])),
           "raw_ctypes_plus_convert": per_call(raw_conv),
           "raw_ctypes": per_call(raw),
           "datetime_now": per_call(lambda: ie._dt.datetime.now())}

    def mut_table_for():
        ins["name"] = "Tom" if ins["name"] != "Tom" else "Ann"
        return ie.table_for(ins)

    def mut_call():
        ins["name"] = "Tom" if ins["name"] != "Tom" else "Ann"
        return ie.interpolate_inserts(ins, s)
    out["after_mutation_call"] = per_call(mut_call, 1000)
    out["after_mutation_table_for"] = per_call(mut_table_for, 1000)
    tt = ie.table_for(ins)

    def upd_only():
        ins["name"] = "Tom" if ins["name"] != "Tom" else "Ann"
        tt.refresh(ins)
    out["refresh_only"] = per_call(upd_only, 1000)
    lib_s, split = [], []
    for _ in range(500):
        upd_only()
        lib_s.append(tt.last_update_native_s)
        split.append(tt.last_update_split_s)
    lib_s.sort()
    out["refresh_library_us_median"] = round(1e6 * lib_s[len(lib_s) // 2], 2)
    out["refresh_pack_us_median"] = round(1e6 * sorted(x[0] for x in split)[len(split) // 2], 2)
    out["refresh_values_us_median"] = round(1e6 * sorted(x[2] for x in split)[len(split) // 2], 2)
    changes = [(0, "name", "Zed")]
    out["update_1_us"] = per_call(lambda: tt.update(changes), 1000)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
