"""Diagnostic (not product): time _ie_pack.pack on a config-5-like store batch (10k states x 5 changes,
the history texts growing each iteration). Usage: python tools/exp/pack_ubench.py new|old|b THREADS; "old" / "b"
load a build of another ie_pack.c variant from tools/exp/pack_old/ or tools/exp/pack_b/ (not kept in the tree)."""
import sys, time, random, importlib.util
which = sys.argv[1]
path = {"old": "tools/exp/pack_old/_ie_pack.cpython-310-x86_64-linux-gnu.so", "b": "tools/exp/pack_b/_ie_pack.cpython-310-x86_64-linux-gnu.so"}.get(which, "/root/repo/interpolation-engine_amd/_ie_pack.cpython-310-x86_64-linux-gnu.so")
spec = importlib.util.spec_from_file_location("_ie_pack", path); P = importlib.util.module_from_spec(spec); spec.loader.exec_module(P)
sys.path.insert(0, "/root/repo")
words = "the knight walks into a dark hall and sees a door to the north there is a faint light you hear steps behind you a guard asks for your name the road is long and cold an old woman sells bread at the gate ask about the castle open the chest look around take the sword go north talk to the guard the wizard smiles and nods é € 😀".split()
rng = random.Random(1)
hist = [" ".join(rng.choice(words) for _ in range(1500)) for _ in range(10000)]
DEL = object()
def render(v, d): return (0, str(v))
for it in range(6):
    changes = []
    for j in range(10000):
        hist[j] = hist[j] + " <action>" + " ".join(rng.choice(words) for _ in range(40))
        changes += [(j, "new_user_input", "look around é"), (j, "maybe_input", "go"), (j, "output", " ".join(rng.choice(words) for _ in range(30))), (j, "history_text_llm", hist[j]), (j, "length_history", it)]
    t = time.perf_counter(); kv, tids, keep = P.pack(changes, 10000, DEL, render, "py", int(sys.argv[2])); dt = time.perf_counter() - t
    del keep
    print(which, it, round(dt * 1e3, 2), "ms", len(hist[0]))
