"""The drop-in mirror in the caller's regime (one string per call, a dict that changes between
tasks), next to the batched path: table build times at 1k / 100k keys, a scalar
interpolate_inserts on an unchanged dict, the same after a mutation (a table rebuild per call),
a 10k-string interpolate_batch, and a 10k-state table set updated in place (one key per state) next
to its rebuild. Prints one JSON object (the GPU box: `python tools/mirror_latency.py`).
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
    # the process's first table build also pays the device's and the library's start-up (context,
    # code objects, the exec's buffers): reported apart, then each size built warm
    d = {"k%d" % i: "value number %d" % i for i in range(1_000)}
    t0 = time.perf_counter()
    pkg.InsertsTable(d).close()
    out["table_build_s_1k_cold_first_in_process"] = round(time.perf_counter() - t0, 4)
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
    # a table set of 10k agent states (config 5's), one key changed per state between two batches:
    # in place (InsertsTableSet.update -> ie_table_set_update) against a rebuild of the set
    from interpolation_engine_amd import workloads as Wk
    defaults = json.load(open(os.path.join(ROOT, "tests", "golden", "config5_stream.json"), encoding="utf-8"))["defaults"]
    states = [Wk.state_inserts(defaults, j) for j in range(10_000)]
    t0 = time.perf_counter()
    tset = pkg.InsertsTableSet(states, clock=(12, 34, 56), mutable=True)
    out["states_10k_build_ms"] = round(1e3 * (time.perf_counter() - t0), 2)
    times, lib_times = [], []
    for it in range(3):
        changes = [(j, "new_user_input", "go north %d %d" % (it, j)) for j in range(len(states))]
        for j, k, v in changes:
            states[j][k] = v
        t0 = time.perf_counter()
        assert tset.update(changes)
        times.append(time.perf_counter() - t0)
        lib_times.append(tset.last_update_native_s)
    out["states_10k_one_key_each_update_ms"] = [round(1e3 * x, 2) for x in times]
    out["states_10k_one_key_each_library_ms"] = [round(1e3 * x, 2) for x in lib_times]
    got = tset.results(["{new_user_input}!"] * 3, [0, 4999, 9999])
    assert got == [states[j]["new_user_input"] + "!" for j in (0, 4999, 9999)], got
    tset.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
