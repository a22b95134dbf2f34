"""Diagnostic: 30 one-key refreshes of a scalar table (run with IE_HOST_TRACE=1: the library's update phases)."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import __graft_entry__ as G
pkg = G.load_package()
ie = pkg.interpolation_engine
ins = ie.VersionedInserts({"k%d" % i: "v%d" % i for i in range(100)})
ins["name"] = "Tom"
s = "Hello {name}"
for i in range(30):
    ins["name"] = "Tom" if i % 2 else "Ann"
    ie.interpolate_inserts(ins, s)
print("done")
