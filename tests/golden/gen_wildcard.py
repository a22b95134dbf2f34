#!/usr/bin/env python3
"""Golden vectors for wildcard match / capture, produced by the REFERENCE's own functions
is_wildcard_match / get_wildcard_matches (py:553-567), imported by path at run time exactly as
gen_golden.py does (nothing from the reference is copied; only the input/output records are
written). Runs only in the build container, where /root/reference exists.

  wildcard_py.jsonl   {"w": wildcard, "s": string, "match": bool, "caps": [...]}

Cases: the wildcard lists of examples/text_adventure.json5 (replace_map at :33-59, the
goto_map / replace_map '|' lists at :131-212, delete_except at :29) against history-like texts
(tags, nested tags, blank-line runs, leading/trailing spaces and newlines, multibyte text), the
regex-special and U+3020 edge cases, and seeded random wildcards over a small alphabet (which
exercise the greedy backtracking and the '$'-before-trailing-newline rule).

Usage:  python tests/golden/gen_wildcard.py [--ref /root/reference/src]
"""
import argparse
import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from gen_golden import import_reference  # noqa: E402

MAP_WILDCARDS = [
    "*<first-output>*</first-output>*", "*<action-output>*</action-output>*", "*<query-output>*</query-output>*",
    "*<query>*</query>*", "*<action>*</action>*", "*  *", "*\n\n\n*", "*\n", "\n*", " *", "* ", "*",
    "false|*", "true|*", "(unset)|*", "*|1", "*|2", "*|3", "*|*", "NULL",
    "scenario", "stage", "history_list", "enable_*", "voice_path", "system_prompt",
]
EDGE_WILDCARDS = ["", "**", "a*", "*a", "a*b*c", "〠", "x〠y", "a.b*", "(*)", "[*]", "\\*", "$*^", "*.*",
                  "é*€", "*😀*", "*\n*\n*", "a**b", "*\n\n", "a", "ab\n"]


def texts(rng):
    words = ["the", "old", "wizard", "é", "€", "😀", "door", "castle", "north", "go", "a", ""]
    out = ["", "\n", " ", "  ", "\n\n\n", "a", "ab", "ab\n", "a\n", "\na", "x\n\n", "false|go north", "true|",
           "(unset)|1", "abc|2", "|", "enable_suggestions", "enable_", "scenario", "stage\n", "NULL", "〠", "x〠y",
           "a.b", "a.bc", "(x)", "[y]", "\\z", "$a^", "é€", "é x €", "😀😀"]
    for _ in range(240):
        parts = []
        for _ in range(rng.randrange(1, 8)):
            r = rng.random()
            if r < 0.25:
                tag = rng.choice(["first-output", "action-output", "query-output", "query", "action"])
                inner = " ".join(rng.choice(words) for _ in range(rng.randrange(0, 6)))
                parts.append("<%s>%s</%s>" % (tag, inner, tag))
            elif r < 0.35:
                parts.append(rng.choice(["\n", "\n\n", "\n\n\n", "\n\n\n\n", "  ", "   ", " "]))
            else:
                parts.append(" ".join(rng.choice(words) for _ in range(rng.randrange(1, 5))))
        out.append("".join(parts))
    return out


def random_cases(rng, n):
    alpha_w = ["a", "b", "*", "*", "\n", " ", "."]
    alpha_s = ["a", "b", "\n", " ", ".", "ab"]
    cases = []
    for _ in range(n):
        w = "".join(rng.choice(alpha_w) for _ in range(rng.randrange(0, 7)))
        s = "".join(rng.choice(alpha_s) for _ in range(rng.randrange(0, 12)))
        cases.append((w, s))
    return cases


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference/src")
    args = ap.parse_args()
    ie = import_reference(args.ref)
    rng = random.Random(0x57AC)
    cases = []
    ts = texts(rng)
    for w in MAP_WILDCARDS + EDGE_WILDCARDS:
        for s in ts[:40] + rng.sample(ts, 40):
            cases.append((w, s))
    cases += random_cases(rng, 3000)
    # strings built to match: captures with every wildcard shape
    for w in MAP_WILDCARDS + EDGE_WILDCARDS:
        for _ in range(6):
            fill = [rng.choice(ts)[:40] for _ in range(w.count("*") + w.count("〠"))]
            s, k = "", 0
            for ch in w:
                if ch in "*〠":
                    s += fill[k]
                    k += 1
                else:
                    s += ch
            cases.append((w, s))
            cases.append((w, s + "\n"))
    seen, n_match = set(), 0
    with open(os.path.join(HERE, "wildcard_py.jsonl"), "w", encoding="utf-8") as f:
        for w, s in cases:
            if (w, s) in seen:
                continue
            seen.add((w, s))
            m = bool(ie.is_wildcard_match(w, s))
            caps = ie.get_wildcard_matches(w, s) if m else []
            n_match += m
            f.write(json.dumps({"w": w, "s": s, "match": m, "caps": caps}, ensure_ascii=False) + "\n")
    print("wildcard_py.jsonl: %d cases, %d matches" % (len(seen), n_match))


if __name__ == "__main__":
    main()
