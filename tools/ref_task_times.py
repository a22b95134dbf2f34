#!/usr/bin/env python3
"""The reference's own per-task cost for the goto_map / replace_map tasks of
examples/text_adventure.json5 (py:1689-1773, through its execute_task, py:1497), on the states of
tests/golden/gen_maps.py, timed on THIS container's CPU (the reference is importable only here, not
on the GPU box). Writes profiles/r03/ref_task_times.json: microseconds per (state, task) for each
task of the program, and over the whole program. tools/task_times.py measures the device path on
the same states and tasks on the GPU box.

Usage:  python tools/ref_task_times.py [--ref /root/reference/src] [--states 240]
"""
import argparse
import asyncio
import copy
import json
import os
import platform
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
sys.path.insert(0, ROOT)
import gen_maps as GM  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference/src")
    ap.add_argument("--states", type=int, default=240)
    args = ap.parse_args()
    ie = GM.import_reference(args.ref)
    ie.log_sink = open(os.devnull, "w")
    text = open(os.path.join(os.path.dirname(args.ref), "examples", "text_adventure.json5"), encoding="utf-8").read()
    program = GM.P.loads(ie.add_line_numbers(text))
    GM.P.label_tasks(program)
    tasks = GM.map_tasks(program)
    defaults = program["default_state"]["inserts"]
    per_task = [0.0] * len(tasks)
    loop = asyncio.new_event_loop()
    for j in range(args.states):
        state = {"order_index": 1, "inserts": GM.make_state(defaults, j), "output": ""}
        for k, t in enumerate(tasks):
            tc = copy.deepcopy(t)
            t0 = time.perf_counter()
            try:
                loop.run_until_complete(ie.execute_task(state, tc, {}, {}, "x"))
            except Exception:  # noqa: BLE001 — an error outcome costs what it cost
                pass
            per_task[k] += time.perf_counter() - t0
    out = {"machine": "%s, %d CPUs (this container; the reference runs single-threaded)" % (platform.processor() or
                                                                                          platform.machine(), os.cpu_count()),
           "states": args.states, "tasks": [t["cmd"] + ":" + str(t.get("line")) for t in tasks],
           "us_per_state_task": [round(1e6 * x / args.states, 1) for x in per_task],
           "us_per_state_program": round(1e6 * sum(per_task) / args.states, 1)}
    os.makedirs(os.path.join(ROOT, "profiles", "r03"), exist_ok=True)
    with open(os.path.join(ROOT, "profiles", "r03", "ref_task_times.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
