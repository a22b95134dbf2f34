#!/usr/bin/env python3
"""Golden vectors for the `unescape` command's transform of its item (py:1660-1667):
recursive_interpolate(inserts, recursive_unescape(item)), generated from the REFERENCE Python
implementation (imported by path at run time, as gen_golden.py does; only the vectors are
written). The point these pin: recursive_interpolate re-enters a whole-string result
(py:1463-1464: `if get_simple_insertkey(x): return recursive_interpolate(inserts,
interpolate_inserts(inserts, x))`), so an item that is a whole-string `{key}` after the unescape
is interpolated again through its value.

  unescape_cmd_py.jsonl   {"t": table index into tables.json, "s": item, "st": status,
                           "out": str result | "value": typed result (JSON)}

Usage:  python tests/golden/gen_unescape_cmd.py [--ref /root/reference/src]
"""
import argparse
import json
import os
import random
import signal
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import gen_golden as GG  # noqa: E402


def run(ie, inserts, s):
    signal.signal(signal.SIGALRM, GG._alarm)
    signal.setitimer(signal.ITIMER_REAL, GG.CASE_TIMEOUT)
    try:
        r = ie.recursive_interpolate(inserts, ie.recursive_unescape(s))
    except GG._Timeout:
        return {"st": "DIVERGED"}
    except ie.InterpolationException:
        return {"st": "E_INTERP"}
    except AssertionError as e:
        return {"st": "E_ASSERT_TYPE" if "trying to interpolate variable" in str(e) else "E_ASSERT_BRACES"}
    except TypeError as e:
        if "unhashable" in str(e):
            return {"st": "E_UNHASHABLE"}
        raise
    except (RecursionError, MemoryError):
        return {"st": "DIVERGED"}
    finally:
        signal.setitimer(signal.ITIMER_REAL, 0)
    if isinstance(r, str):
        return {"st": "OK_STR", "out": r}
    return {"st": "OK_VALUE", "value": r}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference/src")
    ap.add_argument("--seed", type=int, default=20261017)
    args = ap.parse_args()
    ie = GG.import_reference(args.ref)
    tables = json.load(open(os.path.join(HERE, "tables.json"), encoding="utf-8"))
    rng = random.Random(args.seed)
    t0 = tables[0]
    # the named table plus the values the recursion walks into: strings that are references
    # themselves, lists and dicts holding references, scalars returned as they are
    t0 = dict(t0)
    t0.update({"r1": "x {k} y", "r2": "{r1}", "r3": "{b}", "rl": ["{k}", "a{n}", 5, ["{b}"]], "rd": {"{k}": "{n}"},
               "ri": 7, "rf": 2.5, "rn": None, "rt": True, "re": "\\{k\\}", "rmiss": "{nope}", "rbad": "a{b",
               "rsimple": "{{k}}"})
    cases = []
    for k in ["k", "n", "b", "a", "L", "d", "f", "t", "none", "r1", "r2", "r3", "rl", "rd", "ri", "rf", "rn",
              "rt", "re", "rmiss", "rbad", "rsimple", "loop", "tom", "nest", "missing", "esc", "q-1", "HH:MM"]:
        cases += ["\\{%s\\}" % k, "{%s}" % k, "x\\{%s\\}" % k, "\\{%s\\}y" % k, "\\\\{%s\\}" % k,
                  "{\\{%s\\}}" % k, "\\{\\{%s\\}\\}" % k, "\\{%s}" % k]
    cases += GG.named_cases()
    toks = ["\\{", "\\}", "{", "}", "k", "n", "r1", "a", "x", "\\", ".", "é"]
    for _ in range(400):
        cases.append("".join(rng.choice(toks) for _ in range(rng.randint(1, 7))))
    rows = []
    for s in cases:
        rows.append(dict({"t": 0, "s": s}, **run(ie, t0, s)))
    out = {"table": t0, "rows": rows}
    with open(os.path.join(HERE, "unescape_cmd_py.json"), "w", encoding="utf-8") as f:
        json.dump(out, f, ensure_ascii=False, indent=0)
    from collections import Counter
    print("rows:", len(rows), Counter(r["st"] for r in rows))


if __name__ == "__main__":
    main()
