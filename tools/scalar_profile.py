"""Where a scalar interpolate_inserts call spends its time (unchanged dict, after a mutation):
wall times, the refresh/update split, and a cProfile of the mutation loop (GPU box)."""
import cProfile, pstats, sys, os, time, io
sys.path.insert(0, "/root/repo")
import __graft_entry__ as G
G.check_built()
pkg = G.load_package()
ie = pkg.interpolation_engine
ins = ie.VersionedInserts({"k%d" % i: "v%d" % i for i in range(100)})
ins["name"] = "Tom"; ins["kv1"] = "nested"
s = "Hello {name}, item {k7} and {k{k1}}"
def mut():
    ins["name"] = "Tom" if ins["name"] != "Tom" else "Ann"
    return ie.interpolate_inserts(ins, s)
for _ in range(50): mut()
t0 = time.perf_counter()
for _ in range(300): mut()
print("mut us", 1e6 * (time.perf_counter() - t0) / 300)
for _ in range(50): ie.interpolate_inserts(ins, s)
t0 = time.perf_counter()
for _ in range(1000): ie.interpolate_inserts(ins, s)
print("call us", 1e6 * (time.perf_counter() - t0) / 1000)
t = ie.table_for(ins)
t0 = time.perf_counter(); nat = 0
for i in range(300):
    ins["name"] = "X%d" % (i & 1)
    t.refresh(ins); nat += t.last_update_native_s
print("refresh us", 1e6 * (time.perf_counter() - t0) / 300, "native us", 1e6 * nat / 300)
pr = cProfile.Profile(); pr.enable()
for _ in range(300): mut()
pr.disable()
o = io.StringIO(); pstats.Stats(pr, stream=o).sort_stats("tottime").print_stats(25); print(o.getvalue())

# a table set built per map step: build + close of one 100-key dict with brace-bearing values
# (the pre-resolution pass), and the text_adventure map program on one state
d = {"k%d" % i: ("v%d" % i if i % 10 else "<{k%d}>" % (i + 1)) for i in range(100)}
for _ in range(5):
    pkg.InsertsTableSet([d]).close()
t0 = time.perf_counter()
for _ in range(100):
    pkg.InsertsTableSet([d]).close()
print("table set build+close us (10 brace values)", 1e6 * (time.perf_counter() - t0) / 100)
import json as _json
sys.path.insert(0, os.path.join("/root/repo", "tests", "golden"))
from gen_maps import make_state
from interpolation_engine_amd import maps as M
g = _json.load(open("/root/repo/tests/golden/maps_py.json", encoding="utf-8"))
best = None
for _ in range(5):
    st = [make_state(g["defaults"], 3)]
    t0 = time.perf_counter()
    M.run_map_tasks(st, g["tasks"])
    dt = time.perf_counter() - t0
    best = dt if best is None else min(best, dt)
print("map program, one state: us", 1e6 * best)
