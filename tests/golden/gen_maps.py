#!/usr/bin/env python3
"""Golden vectors for goto_map / replace_map (py:1689-1773) from the REFERENCE interpreter.

Every goto_map and replace_map task of examples/text_adventure.json5 (both history replace_maps
with repeat_until_done, the suggestion maps, every goto_map) runs through the reference's own
execute_task (py:1497) on STATES synthetic forked states, and the outcome is recorded: the goto
target, the value replace_map stores, or the error class. The reference module is imported by
path at run time (gen_golden.import_reference); its absent `json5` reads the example through this
repository's JSON5 reader (program.loads), as gen_programs.py does. Only the vectors are written.

The states are workloads.state_inserts(defaults, j, max_entries=12) (deterministic; the test
rebuilds them) with the variation `var(j)` below applied, so the file holds no state text; the
tasks run in program order on each state, replace_map's results carried to the later tasks:

  maps_py.json  {"tasks": [...], "defaults": {...}, "states": N, "results": [[outcome per task]
                 per state]}; an outcome is {"goto": target|null} | {"set": [name, value]} for
                 values up to 256 characters, else {"set": [name, null], "len": L, "fnv": H}
                 (FNV-1a of the UTF-8 bytes) | {"err": class name}; "delete": the program's
                 delete_except tasks on every state and delete edge cases on one state, each
                 outcome {"keys": the remaining keys, sorted} | {"err": class name}

Usage:  python tests/golden/gen_maps.py [--ref /root/reference/src] [--states 240]
"""
import argparse
import asyncio
import copy
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
sys.path.insert(0, ROOT)

from gen_golden import import_reference  # noqa: E402

import __graft_entry__ as G  # noqa: E402

PKG = G.load_package()
from interpolation_engine_amd import program as P  # noqa: E402
from interpolation_engine_amd import workloads as W  # noqa: E402

INPUTS = ["1", "2", "3", "/undo", "/restart", "look around", "", "go {north}", None]
OUTPUTS = ["(unset)", "You see a door.", None]


def var(j):
    """The variation of state j: new_user_input, output, enable_suggestions, suggestions."""
    return {"new_user_input": INPUTS[j % len(INPUTS)], "output": OUTPUTS[(j // 3) % len(OUTPUTS)],
            "enable_suggestions": "true" if (j // 2) % 2 else "false", "suggestions": (j // 5) % 2 == 0}


def make_state(defaults, j):
    ins = W.state_inserts(defaults, j, max_entries=12)
    v = var(j)
    for k in ("new_user_input", "output"):
        if v[k] is None:
            ins.pop(k, None)
        else:
            ins[k] = v[k]
    ins.pop("maybe_input", None)
    ins["enable_suggestions"] = v["enable_suggestions"]
    if v["suggestions"]:
        ins.update({"suggestion_1": "open the gate", "suggestion_2": "ask the {guard}", "suggestion_3": "wait"})
    # what the loop's math commands set before its last goto_maps (text_adventure.json5:264-302)
    n = len(ins["history_list"])
    ins.update({"isodd": n % 2, "length_history": n if j % 7 else 0, "should_summarize": (j % 3) - 1,
                "summarize_ok": (j % 5 > 1) - (j % 5 == 0)})
    return ins


def fnv(s):
    h = 0xCBF29CE484222325
    for b in s.encode("utf-8", "surrogatepass"):
        h = ((h ^ b) * 0x100000001B3) & 0xFFFFFFFFFFFFFFFF
    return h


# Edge cases of the two commands' error order (py:1689-1773) on one small state: an output_name
# that fails (interpolated before replace_map's try, py:1715), failing item leaves and keys with and
# without a 'NULL' map, a key that matches before a failing key, repeat_until_done on captures.
EDGE_STATE = {"a": "apple", "n": 3, "who": "guard", "greet": "hello {who}"}
EDGE_TASKS = [
    {"cmd": "replace_map", "item": "apple pie", "output_name": "{missing_name}",
     "wildcard_maps": [{"apple*": "fruit{1}"}], "traceback_label": "E1"},
    {"cmd": "replace_map", "item": "apple pie", "output_name": "{missing_name}",
     "wildcard_maps": [{"apple*": "x"}, {"NULL": "n"}], "traceback_label": "E2"},
    {"cmd": "replace_map", "item": "x{missing}", "output_name": "out", "wildcard_maps": [{"*": "y"}],
     "traceback_label": "E3"},
    {"cmd": "replace_map", "item": "x{missing}", "output_name": "out", "wildcard_maps": [{"*": "y"}, {"NULL": "nv"}],
     "traceback_label": "E4"},
    {"cmd": "replace_map", "item": "pear", "output_name": "out", "wildcard_maps": [{"{nokey}": "y"}, {"NULL": "nv"}],
     "traceback_label": "E5"},
    {"cmd": "replace_map", "item": "pear", "output_name": "out", "wildcard_maps": [{"p*": "P{1}"}, {"{nokey}": "y"}],
     "traceback_label": "E6"},
    {"cmd": "replace_map", "item": "{a}", "output_name": "res_{n}", "wildcard_maps": [{"app*": "<{1}>"}],
     "traceback_label": "E7"},
    {"cmd": "replace_map", "item": ["{greet}!", {"k{n}": "{a}"}], "output_name": "out",
     "wildcard_maps": [{"hello *": "hi {1}"}, {"*": "[{1}]"}], "traceback_label": "E8"},
    {"cmd": "replace_map", "item": "aaab", "output_name": "out", "repeat_until_done": True,
     "wildcard_maps": [{"a*": "{1}"}], "traceback_label": "E9"},
    {"cmd": "goto_map", "text": "{missing}", "target_maps": [{"x": "t1"}, {"NULL": "tn"}], "traceback_label": "E10"},
    {"cmd": "goto_map", "text": "{missing}", "target_maps": [{"x": "t1"}], "traceback_label": "E11"},
    {"cmd": "goto_map", "text": "abc", "target_maps": [{"{nokey}": "t1"}], "traceback_label": "E12"},
    {"cmd": "goto_map", "text": "{greet}", "target_maps": [{"hello *": "{who}"}], "traceback_label": "E13"},
    # a matched value that fails: the message lists every key of `inserts | extra_inserts` (py:467)
    {"cmd": "replace_map", "item": "apple", "output_name": "out", "wildcard_maps": [{"app*": "{1}{missing_v}"}],
     "traceback_label": "E14"},
    {"cmd": "replace_map", "item": "apple", "output_name": "out", "wildcard_maps": [{"app*": "{greet}{missing_v}"}],
     "traceback_label": "E15"},
]


# delete / delete_except (py:1843-1868) after the task pre-pass (py:1501 interpolates the wildcards)
DELETE_STATE = {"a": "apple", "ab": "x", "b": "banana", "n": 3, "who": "guard", "guard": "g",
                "enable_x": "1", "enable_y": "0", "multi\nline": "m", "k*": "star"}
DELETE_TASKS = [
    {"cmd": "delete", "wildcards": ["a*"], "traceback_label": "D1"},
    {"cmd": "delete_except", "wildcards": ["a*", "enable_*"], "traceback_label": "D2"},
    {"cmd": "delete", "wildcards": ["{who}", "n"], "traceback_label": "D3"},
    {"cmd": "delete_except", "wildcards": [], "traceback_label": "D4"},
    {"cmd": "delete", "wildcards": [], "traceback_label": "D5"},
    {"cmd": "delete", "wildcards": ["*line", "k\\*"], "traceback_label": "D6"},
    {"cmd": "delete", "wildcards": ["{missing}"], "traceback_label": "D7"},
    {"cmd": "delete_except", "wildcards": ["*"], "traceback_label": "D8"},
]


def delete_tasks(program):
    out = []

    def walk(ts):
        for t in ts:
            if isinstance(t, dict) and t.get("cmd") in ("delete", "delete_except"):
                out.append(t)
            if isinstance(t, dict) and isinstance(t.get("tasks"), list):
                walk(t["tasks"])
    walk(program["order"])
    return out


def run_delete(ie, inserts, t):
    """One delete task through the reference's execute_task: the remaining keys (sorted) or the error."""
    state = {"order_index": 1, "inserts": copy.deepcopy(inserts), "output": ""}
    try:
        asyncio.run(ie.execute_task(state, copy.deepcopy(t), {}, {}, "x"))
        return {"keys": sorted(state["inserts"])}
    except Exception as e:  # noqa: BLE001 — the class is the outcome
        return {"err": type(e).__name__}


def run_task(ie, state, t):
    """One task through the reference's execute_task: an outcome record (see the module doc)."""
    try:
        before = dict(state["inserts"])
        r = asyncio.run(ie.execute_task(state, copy.deepcopy(t), {}, {}, "x"))
        if t["cmd"] == "goto_map":
            return {"goto": r["goto_target"] if r else None}
        name = next(k for k in state["inserts"] if k not in before or state["inserts"][k] is not before[k])
        val = state["inserts"][name]
        if isinstance(val, str) and len(val) > 256:
            return {"set": [name, None], "len": len(val), "fnv": fnv(val)}
        return {"set": [name, val]}
    except Exception as e:  # noqa: BLE001 — the class (and the message) is the outcome
        return {"err": type(e).__name__, "msg": str(e)}


def map_tasks(program):
    out = []

    def walk(ts):
        for t in ts:
            if isinstance(t, dict) and t.get("cmd") in ("goto_map", "replace_map"):
                out.append(t)
            if isinstance(t, dict) and isinstance(t.get("tasks"), list):
                walk(t["tasks"])
    walk(program["order"])
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference/src")
    ap.add_argument("--states", type=int, default=240)
    args = ap.parse_args()
    ie = import_reference(args.ref)
    ie.log_sink = open(os.devnull, "w")
    text = open(os.path.join(os.path.dirname(args.ref), "examples", "text_adventure.json5"), encoding="utf-8").read()
    program = P.loads(ie.add_line_numbers(text))
    P.label_tasks(program)
    tasks = map_tasks(program)
    defaults = program["default_state"]["inserts"]
    results = []
    for j in range(args.states):
        row = []
        # the tasks in program order on one evolving state (replace_map's results feed the later
        # maps, e.g. maybe_input -> the suggestions goto_map)
        state = {"order_index": 1, "inserts": make_state(defaults, j), "output": ""}
        for t in tasks:
            try:
                name = ie.interpolate_inserts(state["inserts"], t["output_name"]) if t["cmd"] == "replace_map" else None
                r = asyncio.run(ie.execute_task(state, copy.deepcopy(t), {}, {}, "x"))
                if t["cmd"] == "goto_map":
                    row.append({"goto": r["goto_target"] if r else None})
                else:
                    val = state["inserts"][name]
                    if isinstance(val, str) and len(val) > 256:
                        row.append({"set": [name, None], "len": len(val), "fnv": fnv(val)})
                    else:
                        row.append({"set": [name, val]})
            except Exception as e:  # noqa: BLE001 — the class is the outcome
                row.append({"err": type(e).__name__})
        results.append(row)
    edge = [run_task(ie, {"order_index": 1, "inserts": copy.deepcopy(EDGE_STATE), "output": ""}, t) for t in EDGE_TASKS]
    # the program's delete_except tasks on every state as the loop reaches them (make_state's keys
    # plus what its replace_maps stored), and the delete edge cases on one state
    dtasks = delete_tasks(program)
    dres = [[run_delete(ie, make_state(defaults, j), t) for t in dtasks] for j in range(args.states)]
    dedge = [run_delete(ie, DELETE_STATE, t) for t in DELETE_TASKS]
    out = {"tasks": tasks, "defaults": defaults, "states": args.states, "results": results,
           "edge": {"state": EDGE_STATE, "tasks": EDGE_TASKS, "results": edge},
           "delete": {"tasks": dtasks, "results": dres, "edge_state": DELETE_STATE, "edge_tasks": DELETE_TASKS,
                      "edge_results": dedge}}
    with open(os.path.join(HERE, "maps_py.json"), "w", encoding="utf-8") as f:
        json.dump(out, f, ensure_ascii=False, indent=0)
    from collections import Counter
    print(len(tasks), "tasks;", Counter(k for r in results for o in r for k in o))


if __name__ == "__main__":
    main()
