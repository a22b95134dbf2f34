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
