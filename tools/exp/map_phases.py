"""Where a map step's time goes at 10k states: each goto_map / replace_map task of
tests/golden/maps_py.json through maps.py (as run_map_tasks runs them, one table set), with the
library call timed apart (the ctypes entry wrapped). Prints one JSON line: per task, the step's
wall time and the library call's, in ms."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    import __graft_entry__ as G
    G.check_built()
    pkg = G.load_package()
    from interpolation_engine_amd import maps as M
    IE = pkg.interpolation_engine
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    from gen_maps import make_state
    g = json.load(open(os.path.join(ROOT, "tests", "golden", "maps_py.json"), encoding="utf-8"))
    n = int(os.environ.get("STATES", "10000"))
    L = IE.N.lib()
    spent = {"lib": 0.0}
    for name in ("ie_goto_map", "ie_replace_map"):
        orig = getattr(L, name)

        def wrap(*a, _orig=orig):
            t0 = time.perf_counter()
            try:
                return _orig(*a)
            finally:
                spent["lib"] += time.perf_counter() - t0
        setattr(L, name, wrap)
    out = []
    for rep in range(2):
        st = [make_state(g["defaults"], j % 240) for j in range(n)]
        tset = IE.InsertsTableSet(st)
        rows = []
        for ti, task in enumerate(g["tasks"]):
            fn = M.goto_map_states if task["cmd"] == "goto_map" else M.replace_map_states
            spent["lib"] = 0.0
            prof = None
            if rep and str(ti) in os.environ.get("PROFILE_TASKS", "").split(","):  # cProfile of chosen steps
                import cProfile
                prof = cProfile.Profile()
                prof.enable()
            t0 = time.perf_counter()
            fn(st, task, tables=tset)
            if prof:
                prof.disable()
                import io
                import pstats
                buf = io.StringIO()
                pstats.Stats(prof, stream=buf).sort_stats("tottime").print_stats(25)
                sys.stderr.write("== task %d\n" % ti + buf.getvalue())
            rows.append((task["cmd"][:4], round(1e3 * (time.perf_counter() - t0), 2), round(1e3 * spent["lib"], 2)))
        tset.close()
        out = rows
    print(json.dumps({"states": n, "task_step_ms_lib_ms": out}))


if __name__ == "__main__":
    main()
