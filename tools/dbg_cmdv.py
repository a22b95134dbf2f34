"""Debug helper: the fused views command on the golden items, printing mismatches."""
import sys
sys.path.insert(0, ".")
import numpy as np
import tests.test_gpu_parity as T
from tests.conftest import load_golden

g = load_golden("unescape_cmd_py.json")
strings = [r["s"] for r in g["rows"]]
t = T.PKG.InsertsTable(g["table"], clock=T.CLOCK)
x = T.N.Exec(0)
ref = T._cmd_oracle(T.O.Oracle(g["table"], "py", clock=T.CLOCK), strings)
for vi in (False, True):
    st, res, vid = T._cmd_views(x, t.h, strings, views_input=vi)
    for i in np.flatnonzero(st != ref[0])[:10]:
        print(vi, i, repr(strings[i]), st[i], ref[0][i], res[i], vid[i], ref[3][i])
