"""Where a 10k-state table set's build time goes (Python vs the library): cProfile of
InsertsTableSet(states, mutable=True) over config 5's states. Run on the GPU box."""
import cProfile
import io
import json
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import __graft_entry__ as G
    G.check_built()
    pkg = G.load_package()
    from interpolation_engine_amd import workloads as Wk
    defaults = json.load(open(os.path.join(ROOT, "tests", "golden", "config5_stream.json"), encoding="utf-8"))["defaults"]
    states = [Wk.state_inserts(defaults, j) for j in range(10_000)]
    pkg.InsertsTableSet(states[:100], clock=(12, 34, 56), mutable=True).close()  # warm
    for rep in range(2):
        prof = cProfile.Profile() if rep else None
        t0 = time.perf_counter()
        if prof:
            prof.enable()
        t = pkg.InsertsTableSet(states, clock=(12, 34, 56), mutable=True)
        if prof:
            prof.disable()
        print("build ms", round(1e3 * (time.perf_counter() - t0), 2), flush=True)
        t.close()
    buf = io.StringIO()
    pstats.Stats(prof, stream=buf).sort_stats("tottime").print_stats(15)
    print(buf.getvalue())


if __name__ == "__main__":
    main()
