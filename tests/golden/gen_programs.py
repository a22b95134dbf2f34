#!/usr/bin/env python3
"""Generate program-level golden vectors from the REFERENCE interpreter (configs 1 and 5).

Runs only in the build container (/root/reference never travels to the GPU box). The reference
module is imported by path at run time exactly as gen_golden.py does; its `json5` import is
absent here, so the reference is fed this repository's own JSON5 reader
(interpolation-engine_amd/program.py `loads`) — the verdict's "feed the reference the builder's
own parse". Everything else runs unchanged in the reference: its add_line_numbers (py:2267),
load (py:2283) with validate_program (py:1017), execute_task (py:1497) and recursive_interpolate
(py:1462). Only I/O is stubbed: the InputOutputManager (prompt_toolkit UI) collects writes and
answers user_input with scripted text, and `chat` (the LLM call, py:602) stops the replay.

Writes (JSON data only, no reference source):
  programs_py.json     the reference's (program, state) after load() of every example, and
                       add_line_numbers on edge-case texts
  config1_py.json      examples/hello_world.json5 run to the end: every top-level
                       interpolate_inserts call (content -> result), final state, printed text
  config5_trees.json   the same replay's per-task pre-pass (recursive_interpolate py:1501, and
                       the unescape command's py:1666) of the first 12 states: task tree in,
                       inserts version, tree out (or the error class)
  config5_stream.json  examples/text_adventure.json5 replayed from label '@loop' to the first
                       `chat` for STATES synthetic states: every top-level interpolate_inserts
                       call with the caller (the per-task pre-pass py:1501, or replace_map /
                       goto_map / math internals), the inserts dict it saw (as versions: deltas),
                       and the reference's outcome

Usage:  python tests/golden/gen_programs.py [--ref /root/reference] [--states 24]
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

from gen_golden import CLOCK, import_reference  # noqa: E402

import __graft_entry__ as G  # noqa: E402

PKG = G.load_package()
from interpolation_engine_amd import program as P  # noqa: E402
from interpolation_engine_amd import workloads as W  # noqa: E402


class StopReplay(Exception):
    pass


def outcome(ie, f, *a):
    try:
        r = f(*a)
    except ie.InterpolationException:
        return {"st": "E_INTERP"}
    except AssertionError as e:
        return {"st": "E_ASSERT_TYPE" if "trying to interpolate variable" in str(e) else "E_ASSERT_BRACES"}
    except TypeError as e:
        if "unhashable" in str(e):
            return {"st": "E_UNHASHABLE"}
        raise
    return {"st": "OK", "out": r}


def install_fakes(ie, inputs):
    class FakeIO:
        written = []

        def __init__(self):
            pass

        async def start(self):
            pass

        async def stop(self):
            pass

        async def write(self, text):
            FakeIO.written.append(text)

        async def clear(self):
            FakeIO.written.append("<clear>")

        async def user_input(self, prompt="", default=""):
            await asyncio.sleep(0)
            return inputs.pop(0) if inputs else "look around"

        async def select_index(self, options=None, description="", **k):
            await asyncio.Event().wait()  # waits until the race cancels it

    async def chat(*a, **k):
        raise StopReplay()

    ie.InputOutputManager = FakeIO
    ie.chat = chat
    return FakeIO


class Recorder:
    """Wraps the module-global interpolate_inserts: records depth-0 calls (the nested whole-string
    recursion of py:512/514 is part of one call), the caller, and the inserts dict as versions."""

    def __init__(self, ie, orig):
        self.ie = ie
        self.orig = orig
        self.depth = 0
        self.calls = []
        self.versions = []  # full dicts (JSON-normalised) for delta encoding
        self.deltas = []

    def version_of(self, inserts):
        snap = json.loads(json.dumps(inserts, ensure_ascii=False))
        if self.versions and self.versions[-1] == snap and list(self.versions[-1]) == list(snap):
            return len(self.versions) - 1
        prev = self.versions[-1] if self.versions else {}
        d = {"set": {k: v for k, v in snap.items() if k not in prev or prev[k] != v},
             "del": [k for k in prev if k not in snap]}
        kept = [k for k in prev if k in snap] + [k for k in snap if k not in prev]
        if kept != list(snap):
            d["order"] = list(snap)
        self.versions.append(snap)
        self.deltas.append(d)
        return len(self.versions) - 1

    def __call__(self, inserts, content):
        if self.depth:
            return self.orig(inserts, content)
        caller = sys._getframe(1).f_code.co_name
        v = self.version_of(inserts)
        self.depth += 1
        try:
            rec = outcome(self.ie, self.orig, inserts, content)
        finally:
            self.depth -= 1
        row = {"v": v, "by": caller, "s": content, "st": rec["st"]}
        if rec["st"] == "OK":
            r = rec["out"]
            if isinstance(r, str) and not P._simple_key(content.replace("\\{", ".〠").replace("\\}", "〠.")):
                row["out"] = r
            else:  # typed (whole-string) result: the keys whose value is that object
                row["st"] = "OK_VALUE"
                row["vkeys"] = [k for k, x in inserts.items() if x is r]
                if not row["vkeys"]:
                    row["value"] = r  # a fresh object (the clock keys)
            if row["st"] == "OK":
                row["st"] = "OK_STR"
        self.calls.append(row)
        if rec["st"] != "OK":
            raise {"E_INTERP": self.ie.InterpolationException}.get(rec["st"], AssertionError)("recorded failure")
        return rec["out"]


class TreeRecorder:
    """Wraps the module-global recursive_interpolate: records the depth-0 calls (the per-task
    pre-pass py:1501 and the unescape command's py:1666) with the task tree passed in, the inserts
    version the call saw (shared with the Recorder) and the tree the reference returned."""

    def __init__(self, ie, orig, rec):
        self.ie, self.orig, self.rec = ie, orig, rec
        self.depth = 0
        self.trees = []

    def __call__(self, inserts, x):
        if self.depth:
            return self.orig(inserts, x)
        caller = sys._getframe(1).f_code.co_name
        v = self.rec.version_of(inserts)
        tree = json.loads(json.dumps(x, ensure_ascii=False))
        self.depth += 1
        try:
            r = self.orig(inserts, x)
        except self.ie.InterpolationException:
            self.trees.append({"v": v, "by": caller, "x": tree, "st": "E_INTERP"})
            raise
        except AssertionError:
            self.trees.append({"v": v, "by": caller, "x": tree, "st": "E_ASSERT"})
            raise
        finally:
            self.depth -= 1
        self.trees.append({"v": v, "by": caller, "x": tree, "st": "OK", "out": json.loads(json.dumps(r, ensure_ascii=False))})
        return r


async def drive(ie, program, state, stop_at_chat=True, max_tasks=400):
    completion_args = program.get("completion_args", {})
    named = program.get("named_tasks", {})
    order = program["order"]
    n = 0
    while state["order_index"] <= len(order):
        task = order[state["order_index"] - 1]
        result = await ie.execute_task(state, task, completion_args, named, task["traceback_label"])
        if result is None:
            state["order_index"] += 1
        else:
            state["order_index"] = 2 + min(i for i in range(len(order)) if order[i]["cmd"] == "label"
                                           and order[i]["name"] == result["goto_target"])
        n += 1
        if n > max_tasks:
            raise RuntimeError("replay did not reach a chat")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("--states", type=int, default=24)
    args = ap.parse_args()
    ie = import_reference(os.path.join(args.ref, "src"))
    ie.json5.loads = P.loads
    ie.log_sink = open(os.devnull, "w")
    ex = os.path.join(args.ref, "examples")
    orig = ie.interpolate_inserts

    # ---- A: load() of every example, add_line_numbers edge cases ----
    progs = {}
    for f in sorted(os.listdir(ex)):
        try:
            ie.disk_program_hash = None
            program, state = ie.load(os.path.join(ex, f))
            progs[f] = {"program": program, "state": state}
        except AssertionError as e:
            progs[f] = {"error": "AssertionError", "msg": str(e)[:200]}
    texts = ["{cmd:'print', text:'x'}", "{ cmd : \"set\" , item:1}", "{'cmd':'a'}\n{\"cmd\":'b' }",
             "x = {cmd:'it\\'s'},\r\n{cmd:'q\"'}", "{command:'x'}", "{cmd:'a'} {cmd:'b'}", "{cmd: 'x' ,}",
             "line1\nline2 {cmd:'z'} {cmd:'w'}"]
    lines = [{"in": t, "out": ie.add_line_numbers(t)} for t in texts]
    with open(os.path.join(HERE, "programs_py.json"), "w", encoding="utf-8") as fh:
        json.dump({"programs": progs, "add_line_numbers": lines}, fh, ensure_ascii=False, indent=0)

    # ---- B: config 1, hello_world to the end ----
    rec = Recorder(ie, orig)
    ie.interpolate_inserts = rec
    io = install_fakes(ie, [])
    ie.disk_program_hash = None
    program, state = ie.load(os.path.join(ex, "hello_world.json5"))
    asyncio.run(drive(ie, program, state, stop_at_chat=False))
    with open(os.path.join(HERE, "config1_py.json"), "w", encoding="utf-8") as fh:
        json.dump({"calls": rec.calls, "state": state, "written": io.written, "stdout": state["output"].strip()},
                  fh, ensure_ascii=False, indent=0)
    print("config 1:", len(rec.calls), "interpolations, stdout %r" % state["output"].strip())

    # ---- C: config 5, text_adventure from '@loop' to the first chat, per synthetic state ----
    ie.disk_program_hash = None
    program0, state0 = ie.load(os.path.join(ex, "text_adventure.json5"))
    defaults = copy.deepcopy(state0["inserts"])
    loop_at = 1 + next(i for i, t in enumerate(program0["order"]) if t["cmd"] == "label" and t["name"] == "@loop")
    out = {"defaults": defaults, "clock": CLOCK, "states": []}
    trees = {"clock": CLOCK, "states": []}
    orig_ri = ie.recursive_interpolate
    total = 0
    for j in range(args.states):
        syn = W.state_inserts(defaults, j, max_entries=8 if j < args.states - 4 else 36)  # 4 long-history states
        state = copy.deepcopy(state0)
        state["inserts"] = {k: syn[k] for k in list(defaults) + ["scenario", "stage", "history_list"]}
        state["order_index"] = loop_at
        program = copy.deepcopy(program0)
        rec = Recorder(ie, orig)
        ie.interpolate_inserts = rec
        tr = TreeRecorder(ie, orig_ri, rec)
        ie.recursive_interpolate = tr
        install_fakes(ie, [syn["new_user_input"], "look around"])
        try:
            asyncio.run(drive(ie, program, state))
            raise RuntimeError("no chat reached")
        except StopReplay:
            pass
        ie.recursive_interpolate = orig_ri
        out["states"].append({"stage": syn["stage"], "deltas": rec.deltas, "calls": rec.calls})
        if j < 12:  # the per-task pre-pass trees of the first 12 states (file size)
            trees["states"].append({"stage": syn["stage"], "deltas": rec.deltas, "trees": tr.trees})
        total += len(rec.calls)
    ie.interpolate_inserts = orig
    with open(os.path.join(HERE, "config5_stream.json"), "w", encoding="utf-8") as fh:
        json.dump(out, fh, ensure_ascii=False, separators=(",", ":"))
    with open(os.path.join(HERE, "config5_trees.json"), "w", encoding="utf-8") as fh:
        json.dump(trees, fh, ensure_ascii=False, separators=(",", ":"))
    print("config 5 trees: %d bytes" % os.path.getsize(os.path.join(HERE, "config5_trees.json")))
    print("config 5: %d states, %d calls, %d bytes" % (args.states, total,
                                                      os.path.getsize(os.path.join(HERE, "config5_stream.json"))))


if __name__ == "__main__":
    main()
