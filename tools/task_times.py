#!/usr/bin/env python3
"""The device path's per-task cost for the goto_map / replace_map tasks of
examples/text_adventure.json5 (interpolation-engine_amd/maps.py: one device batch per step of the
reference's loop over every state still running it), on tests/golden/gen_maps.py's states, for
1, 240 and 10,000 forked states: microseconds per (state, task), next to the reference's own cost
timed on the CPU by tools/ref_task_times.py (profiles/r03/ref_task_times.json). Prints one JSON line.
Run on the GPU box:  python tools/task_times.py
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import __graft_entry__ as G
    G.check_built()
    G.load_package()
    from interpolation_engine_amd import maps as M
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    from gen_maps import make_state  # the states the reference's vectors were made on
    g = json.load(open(os.path.join(ROOT, "tests", "golden", "maps_py.json"), encoding="utf-8"))
    out = {"tasks": len(g["tasks"])}
    for n in (1, 240, 10_000):
        states = [make_state(g["defaults"], j % 240) for j in range(n)]
        per_task = [0.0] * len(g["tasks"])
        for rep in range(2):  # the first pass warms the library (execs, code objects)
            st = [dict(s) for s in states]
            for k, task in enumerate(g["tasks"]):
                fn = M.goto_map_states if task["cmd"] == "goto_map" else M.replace_map_states
                t0 = time.perf_counter()
                got = fn(st, task)
                dt = time.perf_counter() - t0
                if rep:
                    per_task[k] += dt
                if task["cmd"] == "replace_map":
                    for j, r in enumerate(got):
                        if not isinstance(r, BaseException):
                            st[j][r[0]] = r[1]
        # the whole program through run_map_tasks (one table set per stretch of unchanged states)
        best = None
        for rep in range(2):
            st = [dict(s) for s in states]
            prof = None
            # where the host time goes: IE_TASK_PROFILE (10k states) or IE_TASK_PROFILE_N=<states>
            pn = int(os.environ.get("IE_TASK_PROFILE_N") or (10_000 if os.environ.get("IE_TASK_PROFILE") else 0))
            if rep and n == pn:
                import cProfile
                prof = cProfile.Profile()
                prof.enable()
            t0 = time.perf_counter()
            M.run_map_tasks(st, g["tasks"])
            dt = time.perf_counter() - t0
            if prof:
                prof.disable()
                import io
                import pstats
                buf = io.StringIO()
                pstats.Stats(prof, stream=buf).sort_stats("tottime").print_stats(40)
                sys.stderr.write(buf.getvalue())
            best = dt if best is None else min(best, dt)
        out.setdefault("rebuilds", {})["states_%d" % n] = list(M.REBUILDS)
        M.REBUILDS.clear()
        out["states_%d" % n] = {"us_per_state_task": [round(1e6 * x / n, 2) for x in per_task],
                                "us_per_state_program_task_by_task": round(1e6 * sum(per_task) / n, 2),
                                "us_per_state_program": round(1e6 * best / n, 2)}
    ref = os.path.join(ROOT, "profiles", "r03", "ref_task_times.json")
    if os.path.exists(ref):
        r = json.load(open(ref))
        out["reference_cpu_us_per_state_program"] = r["us_per_state_program"]
        for n in (1, 240, 10_000):
            out["states_%d" % n]["vs_reference"] = round(r["us_per_state_program"] / out["states_%d" % n]["us_per_state_program"], 3)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
