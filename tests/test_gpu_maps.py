"""goto_map / replace_map (py:1689-1773) over batches of forked states on the device, against the
reference's own execute_task run on the same states (tests/golden/gen_maps.py -> maps_py.json):
every goto_map and replace_map task of examples/text_adventure.json5, applied in program order to
240 synthetic states (both history replace_maps with repeat_until_done, the suggestion maps with
captures and 'NULL', every goto_map). One device batch per task over all states."""
import pytest

import __graft_entry__ as G
from tests.conftest import load_golden

pytestmark = pytest.mark.gpu

G.build()
PKG = G.load_package()
from interpolation_engine_amd import maps as M  # noqa: E402
from interpolation_engine_amd import workloads as W  # noqa: E402

INPUTS = ["1", "2", "3", "/undo", "/restart", "look around", "", "go {north}", None]
OUTPUTS = ["(unset)", "You see a door.", None]


def make_state(defaults, j):
    """tests/golden/gen_maps.py make_state (the same deterministic states)."""
    ins = W.state_inserts(defaults, j, max_entries=12)
    v = {"new_user_input": INPUTS[j % len(INPUTS)], "output": OUTPUTS[(j // 3) % len(OUTPUTS)],
         "enable_suggestions": "true" if (j // 2) % 2 else "false", "suggestions": (j // 5) % 2 == 0}
    for k in ("new_user_input", "output"):
        if v[k] is None:
            ins.pop(k, None)
        else:
            ins[k] = v[k]
    ins.pop("maybe_input", None)
    ins["enable_suggestions"] = v["enable_suggestions"]
    if v["suggestions"]:
        ins.update({"suggestion_1": "open the gate", "suggestion_2": "ask the {guard}", "suggestion_3": "wait"})
    n = len(ins["history_list"])
    ins.update({"isodd": n % 2, "length_history": n if j % 7 else 0, "should_summarize": (j % 3) - 1,
                "summarize_ok": (j % 5 > 1) - (j % 5 == 0)})
    return ins


def fnv(s):
    h = 0xCBF29CE484222325
    for b in s.encode("utf-8", "surrogatepass"):
        h = ((h ^ b) * 0x100000001B3) & 0xFFFFFFFFFFFFFFFF
    return h


def _check(want, got):
    if "err" in want:
        return isinstance(got, BaseException) and type(got).__name__ == want["err"]
    if isinstance(got, BaseException):
        return False
    if "goto" in want:
        return (got["goto_target"] if got else None) == want["goto"]
    name, value = got
    if want["set"][0] != name:
        return False
    if "fnv" in want:
        return isinstance(value, str) and len(value) == want["len"] and fnv(value) == want["fnv"]
    return value == want["set"][1] and type(value) == type(want["set"][1])


def test_text_adventure_maps_match_reference():
    g = load_golden("maps_py.json")
    states = [make_state(g["defaults"], j) for j in range(g["states"])]
    bad = []
    for k, task in enumerate(g["tasks"]):
        fn = M.goto_map_states if task["cmd"] == "goto_map" else M.replace_map_states
        got = fn(states, task)
        for j, r in enumerate(got):
            if not _check(g["results"][j][k], r):
                bad.append((k, task["cmd"], task.get("text", task.get("item")), j, g["results"][j][k],
                            repr(r)[:200]))
            if task["cmd"] == "replace_map" and not isinstance(r, BaseException):
                states[j][r[0]] = r[1]  # set_interpdata: the later tasks see it
    assert not bad, (len(bad), bad[:6])


def test_run_map_tasks_matches_reference():
    """The same program through run_map_tasks (table sets shared while the states do not change;
    each map value interpolated against the captures and the keys it can reach)."""
    g = load_golden("maps_py.json")
    states = [make_state(g["defaults"], j) for j in range(g["states"])]
    outs = M.run_map_tasks(states, g["tasks"])
    bad = [(k, j) for k, got in enumerate(outs) for j, r in enumerate(got) if not _check(g["results"][j][k], r)]
    assert not bad, (len(bad), bad[:6])


def test_single_state_entry_points():
    """goto_map / replace_map for one state (the reference's call regime) agree with the batch."""
    g = load_golden("maps_py.json")
    ins = make_state(g["defaults"], 1)
    for k, task in enumerate(g["tasks"][:8]):
        want = g["results"][1][k]
        if task["cmd"] == "goto_map":
            if "err" in want:
                with pytest.raises(AssertionError):
                    M.goto_map(ins, task)
            else:
                r = M.goto_map(ins, task)
                assert (r["goto_target"] if r else None) == want["goto"]
        elif "err" not in want:
            M.replace_map(ins, task)
            assert _check(want, (want["set"][0], ins[want["set"][0]]))


def test_error_order_edges_match_reference():
    """Reference-generated edge cases (tests/golden/gen_maps.py EDGE_TASKS): an output_name that
    fails raises its InterpolationException whatever 'NULL' says (py:1715 is before the try), item
    leaves and keys that fail with and without 'NULL', a key matching before a failing key,
    repeat_until_done over captures, goto_map's text / key failures; a matched value that fails.
    Errors compare by class and message (the message lists the keys of the table a lookup missed
    in, py:467, and replace_map embeds it, py:1767)."""
    import copy
    e = load_golden("maps_py.json")["edge"]
    bad = []
    for task, want in zip(e["tasks"], e["results"]):
        fn = M.goto_map_states if task["cmd"] == "goto_map" else M.replace_map_states
        got = fn([copy.deepcopy(e["state"])], task)[0]
        if not _check(want, got) or ("msg" in want and str(got) != want["msg"]):
            bad.append((task["traceback_label"], want, repr(got)[:300]))
    assert not bad, bad


def test_delete_except_of_the_program_matches_reference():
    """text_adventure.json5's delete_except tasks (:29, :63) on every state, one library call per task
    over all states (ie_delete_keys: every key of every state in one k_wildcard launch, the keys
    removed from the device table set in place), against the reference's execute_task."""
    g = load_golden("maps_py.json")
    d = g["delete"]
    bad = []
    for k, task in enumerate(d["tasks"]):
        states = [make_state(g["defaults"], j) for j in range(g["states"])]
        tset = M.IE.InsertsTableSet(states, mutable=True)
        try:
            gone = M.delete_states(states, task, tables=tset)
            # the device copy agrees with the dicts: every remaining key resolves, no deleted one does
            probe = [("{%s}" % kk, j) for j, st in enumerate(states) for kk in list(st)[:3]]
            probe += [("{%s}" % kk, j) for j, ks in enumerate(gone) for kk in ks[:2]]
            res = tset.results([p for p, _ in probe], [j for _, j in probe])
        finally:
            tset.close()
        for j, st in enumerate(states):
            if sorted(st) != d["results"][j][k]["keys"]:
                bad.append((k, j, sorted(st), d["results"][j][k]))
        for (p, j), r in zip(probe, res):
            key = p[1:-1]
            if (key in states[j]) == isinstance(r, BaseException):
                bad.append(("device", j, key, repr(r)[:80]))
    assert not bad, (len(bad), bad[:6])


def test_delete_edges_match_reference():
    """delete / delete_except edge cases (tests/golden/gen_maps.py DELETE_TASKS): interpolated
    wildcards, empty lists, DOTALL groups across a newline, a wildcard that fails to interpolate."""
    import copy
    d = load_golden("maps_py.json")["delete"]
    bad = []
    for task, want in zip(d["edge_tasks"], d["edge_results"]):
        st = copy.deepcopy(d["edge_state"])
        got = M.delete_states([st], task)[0]
        if "err" in want:
            ok = isinstance(got, BaseException) and type(got).__name__ == want["err"]
        else:
            ok = not isinstance(got, BaseException) and sorted(st) == want["keys"]
        if not ok:
            bad.append((task["traceback_label"], want, repr(got)[:200], sorted(st)))
    assert not bad, bad
