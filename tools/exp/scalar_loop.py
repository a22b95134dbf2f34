"""Diagnostic: 2000 scalar interpolate_inserts calls (for a rocprofv3 runtime trace of one call's HIP API sequence)."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import __graft_entry__ as G
pkg = G.load_package()
ie = pkg.interpolation_engine
ins = ie.VersionedInserts({"k%d" % i: "v%d" % i for i in range(100)})
ins["name"] = "Tom"
ins["kv1"] = "nested"
s = "Hello {name}, item {k7} and {k{k1}}"
for _ in range(2000):
    ie.interpolate_inserts(ins, s)
print("done")
