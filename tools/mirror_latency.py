"""The drop-in mirror in the caller's regime (one string per call, a dict that changes between
tasks), next to the batched path: table build times at 1k / 100k keys, a scalar
interpolate_inserts on an unchanged dict, the same after a mutation (a table rebuild per call),
and a 10k-string interpolate_batch. Prints one JSON object (the GPU box: `python tools/mirror_latency.py`).
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def per_call(fn, n):
    fn()  # warm
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    return (time.perf_counter() - t0) / n


def main():
    import __graft_entry__ as G
    G.check_built()
    pkg = G.load_package()
    ie = pkg.interpolation_engine
    out = {}
    for nkeys in (1_000, 100_000):
        d = {"k%d" % i: "value number %d" % i for i in range(nkeys)}
        t0 = time.perf_counter()
        t = pkg.InsertsTable(d)
        out["table_build_s_%dk" % (nkeys // 1000)] = round(time.perf_counter() - t0, 4)
        t.close()
    ins = ie.VersionedInserts({"k%d" % i: "v%d" % i for i in range(100)})
    ins["name"] = "Tom"
    s = "Hello {name}, item {k7} and {k{k1}}"
    ins["kv1"] = "nested"
    out["scalar_call_us"] = round(1e6 * per_call(lambda: ie.interpolate_inserts(ins, s), 2000), 1)

    def mutate_and_call():
        ins["name"] = "Tom" if ins["name"] != "Tom" else "Ann"
        return ie.interpolate_inserts(ins, s)
    out["scalar_call_after_mutation_us"] = round(1e6 * per_call(mutate_and_call, 300), 1)
    strings = ["line %d: {name} has {k%d}" % (j, j % 100) for j in range(10_000)]
    dt = per_call(lambda: ie.interpolate_batch(ins, strings), 20)
    out["batch_10k_ms"] = round(1e3 * dt, 3)
    out["batch_per_string_us"] = round(1e6 * dt / len(strings), 3)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
