"""Configs 1 and 5 on the device, against what the reference interpreter did (tests/golden/
gen_programs.py): hello_world through the runner's per-task pre-pass, and the text_adventure
loop's recorded interpolation stream over a table set (one device table per inserts version)."""
import numpy as np
import pytest

import __graft_entry__ as G
from tests.conftest import load_golden
from tests.test_programs import rebuild_versions

pytestmark = pytest.mark.gpu

G.build()
PKG = G.load_package()
N = PKG._native
from interpolation_engine_amd import program as P  # noqa: E402


def test_config1_hello_world_runs_through_the_device():
    ref = load_golden("programs_py.json")["programs"]["hello_world.json5"]
    c1 = load_golden("config1_py.json")
    program, state = ref["program"], dict(ref["state"], inserts=dict(ref["state"]["inserts"]))
    seen = []

    def resolve(inserts, task):
        out = PKG.recursive_interpolate(inserts, task)
        PKG.interpolation_engine._map_strings(task, lambda ss: seen.extend(ss) or ss)
        return out

    written = []
    stdout = P.Runner(program, state, resolve=resolve, write=written.append).run()
    assert stdout == c1["stdout"] == "Hello, world!"
    assert sorted(seen) == sorted(c["s"] for c in c1["calls"])  # the same 7 interpolations
    assert state == c1["state"]


def _stream_batch(c5, first_state=0, n_states=None):
    """The recorded calls as one table-set batch: table = (state, inserts version)."""
    states = c5["states"][first_state:][:n_states]
    tables, starts, items = [], [], []
    for st in states:
        vs = rebuild_versions(st["deltas"])
        starts.append(len(tables))
        tables.extend(vs)
        for c in st["calls"]:
            items.append((starts[-1] + c["v"], c))
    return tables, items


def test_config5_recorded_stream_matches_reference(fail_commit):
    c5 = load_golden("config5_stream.json")
    tables, items = _stream_batch(c5)
    tset = PKG.InsertsTableSet(tables, clock=tuple(c5["clock"]))
    got = tset.run([c["s"] for _, c in items], [t for t, _ in items])
    bad = []
    for (t, c), (st, payload) in zip(items, got):
        name = N.STATUS_NAMES[st]
        want = c["st"]
        ok = name == want
        if ok and want == "OK_STR":
            ok = payload == c["out"]
        if ok and want == "OK_VALUE":
            keys = tset.table_keys(t)
            ok = payload - tset.starts[t] in [keys.index(k) for k in c["vkeys"]] if c["vkeys"] else \
                tset.value(payload) == c["value"]
        if not ok:
            bad.append((t, c, name, payload))
    assert not bad, (len(bad), bad[:3])
    assert len(items) > 4000 and max(len(c.get("out", "")) for _, c in items) > 2000  # multi-KB chat content


def test_config5_prepass_of_one_state_is_recursive_interpolate():
    """The per-task pre-pass calls of one state (py:1501) replayed through the mirror's batched
    recursive_interpolate give the same strings."""
    c5 = load_golden("config5_stream.json")
    st = c5["states"][0]
    vs = rebuild_versions(st["deltas"])
    for c in st["calls"]:
        if c["by"] != "recursive_interpolate" or c["st"] != "OK_STR":
            continue
        assert PKG.interpolate_batch(vs[c["v"]], [c["s"]])[0] == c["out"]


@pytest.fixture(params=["0", "1"], ids=["chain-fail-exact", "chain-fail-commit"])
def fail_commit(request, monkeypatch):
    monkeypatch.setenv("IE_FAIL_COMMIT", request.param)
    PKG.interpolation_engine.get_exec(0).set_option(N.OPT_FAIL_COMMIT, int(request.param))
    yield request.param
    PKG.interpolation_engine.get_exec(0).set_option(N.OPT_FAIL_COMMIT, -1)


def test_config5_prepass_trees_of_all_states_in_one_batch():
    """The per-task pre-pass (recursive_interpolate, py:1501) of every recorded state of the
    text_adventure loop, tree for tree against what the reference returned (gen_programs.py ->
    config5_trees.json), all states' trees in ONE device batch (recursive_interpolate_states)."""
    g = load_golden("config5_trees.json")
    states, xs, want = [], [], []
    for st in g["states"]:
        vs = rebuild_versions(st["deltas"])
        for t in st["trees"]:
            states.append(vs[t["v"]])
            xs.append(t["x"])
            want.append(t)
    got = PKG.recursive_interpolate_states(states, xs, clock=tuple(g["clock"]))
    bad = []
    for w, r in zip(want, got):
        if w["st"] == "OK":
            ok = not isinstance(r, BaseException) and r == w["out"]
        elif w["st"] == "E_INTERP":
            ok = isinstance(r, PKG.InterpolationException)
        else:
            ok = isinstance(r, AssertionError)
        if not ok:
            bad.append((w["x"], w["st"], repr(r)[:200]))
    assert not bad, (len(bad), bad[:3])
    assert len(want) >= 200


def test_errors_come_in_the_walk_order():
    """py:1462-1494 walks a list in order: a missing key in an earlier leaf is raised before the
    loop command's get_interpdata (py:1483-1488) of a later element, and a failing state does not
    fail the other states of the batch."""
    inserts = {"name": "tom"}
    x = ["{missing_a}", {"cmd": "for", "tasks": "{missing_b}"}]
    with pytest.raises(PKG.InterpolationException) as e:
        PKG.recursive_interpolate(inserts, x)
    assert "missing_a" in str(e.value) and "missing_b" not in str(e.value)
    # the loop command's lookup first when it comes first
    with pytest.raises(PKG.InterpolationException) as e:
        PKG.recursive_interpolate(inserts, [{"cmd": "for", "tasks": "{missing_b}"}, "{missing_a}"])
    assert "missing_b" in str(e.value)
    got = PKG.recursive_interpolate_states([inserts, inserts], [x, ["{name}"]])
    assert isinstance(got[0], PKG.InterpolationException) and got[1] == ["tom"]
