"""The scalar mirror call under one IE_SMALL_ZC mode (set in the environment before the library
loads): best of five 2,000-call runs on an unchanged dict and of five 300-call runs after a mutation
(tools/mirror_latency.py's calls). Prints one JSON line."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def per_call(fn, n):
    fn()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    return (time.perf_counter() - t0) / n


def main():
    import __graft_entry__ as G
    G.check_built()
    ie = G.load_package().interpolation_engine
    ins = ie.VersionedInserts({"k%d" % i: "v%d" % i for i in range(100)})
    ins["name"] = "Tom"
    ins["kv1"] = "nested"
    s = "Hello {name}, item {k7} and {k{k1}}"
    assert ie.interpolate_inserts(ins, s) == "Hello Tom, item v7 and nested"

    def mutate_and_call():
        ins["name"] = "Tom" if ins["name"] != "Tom" else "Ann"
        return ie.interpolate_inserts(ins, s)
    a = [per_call(lambda: ie.interpolate_inserts(ins, s), 2000) for _ in range(5)]
    b = [per_call(mutate_and_call, 300) for _ in range(5)]
    print(json.dumps({"zc": os.environ.get("IE_SMALL_ZC", "default"),
                      "scalar_call_us": [round(1e6 * x, 1) for x in a],
                      "after_mutation_us": [round(1e6 * x, 1) for x in b]}))


if __name__ == "__main__":
    main()
