#!/usr/bin/env python3
"""Golden vectors for get_interpdata's inserts-directory fallback (py:452-461), produced by the
REFERENCE's interpolate_inserts with its module global `inserts_dir` pointed at a temporary
directory (imported by path at run time as gen_golden.py does; nothing is copied). The `json5`
package the reference reads `<key>.json5` with is absent here, so the reference is given the
builder's own JSON5 reader (interpolation-engine_amd/program.py `loads`) under that name.

  inserts_dir_py.json  {"files": {relative path: content}, "inserts": {...}, "cases": [{"s", "st",
                       "out" | "value"}]}   (the test recreates the directory from "files")

Usage:  python tests/golden/gen_inserts_dir.py [--ref /root/reference/src]
"""
import argparse
import json
import os
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
from gen_golden import import_reference  # noqa: E402

FILES = {
    "greet.json5": "{msg: 'hi {name}', n: 3}",
    "title.json5": "'The {adj} tower'",
    "count.json5": "42",
    "list.json5": "['a', 'b', 7]",
    "plain": "  Plain text with {braces} and \\\\ a backslash\n\n",
    "both.json5": "'from json5'",
    "both": "from plain",
    "over": "from the directory",
    "sub/nested.json5": "'deep'",
    "sub/leaf": "leaf text",
    "x.json5": "'x as json5'",
    "ARG1": "never read",
    "ARG\u00b2": "never read: str.isdigit() is true for a superscript two",
    "ARG\u0663": "never read: an Arabic-Indic digit three",
    "ARGx": "ARGx is not an argument key",
    "empty": "",
    "unicode": "héllo 😀 〠",
    "q-42": "forty-two",
    "keyname": "count",
    "wrapped.json5": "'{count}'",
    "dotted.name": "a dotted file",
    "spaces key": "with spaces",
}
INSERTS = {"name": "Tom", "adj": "tall", "over": "from the inserts", "k": "keyname", "n": 5}
CASES = [
    "{greet}", "x{greet}y", "{title}", "a {title} b", "{count}", "n={count}", "{list}", "L={list}",
    "{plain}", "[{plain}]", "{both}", "<{both}>", "{over}", "{sub/nested}", "{sub/leaf}", "({sub/leaf})",
    "{x.json5}", "{x}", "{ARG1}", "{ARG2}", "{ARG\u00b2}", "{ARG\u0663}", "{ARGx}", "a {ARG\u00b2} b", "{missing}", "{missing/x}", "{sub/missing}", "{empty}", "[{empty}]",
    "{unicode}", "u={unicode}", "{q-{count}}", "{q-{n}}", "{{k}}", "{{keyname}}", "{wrapped}", "w={wrapped}",
    "{dotted.name}", "{spaces key}", "{name} and {count} and {plain}", "\\{count\\} {count}", "{n}{count}{n}",
    "{HH:MM}", "{}", "no refs at all", "{name}",
]


# keys that are not canonical relative file names (os.path.join may leave the directory, py:455-459)
# and files the reference cannot read: the directory is <base>/dir, these files sit in <base>
OUTSIDE_FILES = {"outside": "an outside {name} file", "outside_j.json5": "'outside json5'", "dir2/leaf": "second dir"}
BAD_FILES = {"binary": "fffe00206e6f74207574662d38", "broken.json5": "7b756e7465726d696e617465643a20"}  # hex
OUTSIDE_CASES = ["{../outside}", "a{../outside}b", "{../outside_j}", "{../nope}", "x{../nope}y", "{sub/../count}",
                 "{./over}", "{sub//leaf}", "{../dir2/leaf}", "{../dir/plain}", "{binary}", "x{binary}y", "{broken}",
                 "{q-{../nope}}", "{sub}", "x{sub}y", "{binary}{missing}", "{missing}{binary}", "{binary}{sub}",
                 "{sub}{count}",
                 # keys built from looked-up values that leave the directory (the device records them)
                 "{{up}/outside}", "x{{up}/nope}y", "<{{up}/dir2/leaf}>", "{{up}/{sub_k}}", "{{up}/outside_j}"]
# the values those keys are built from (added to the inserts of the outside cases only)
OUTSIDE_INSERTS = {"up": "..", "sub_k": "dir"}


def classify(ie, inserts, s, other_errors=False):
    try:
        r = ie.interpolate_inserts(inserts, s)
    except ie.InterpolationException:
        return {"st": "E_INTERP"}
    except AssertionError as e:
        return {"st": "E_ASSERT_TYPE" if "trying to interpolate variable" in str(e) else "E_ASSERT_BRACES"}
    except TypeError as e:
        if "unhashable" in str(e):
            return {"st": "E_UNHASHABLE"}
        raise
    except Exception as e:  # noqa: BLE001 — a file the reference could not read (its own error)
        if not other_errors:
            raise
        return {"st": "RAISES", "exc": type(e).__name__}
    protected = s.replace("\\{", ".〠").replace("\\}", "〠.")
    if ie.get_simple_insertkey(protected):
        return {"st": "OK_VALUE", "value": r}
    return {"st": "OK_STR", "out": r}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference/src")
    args = ap.parse_args()
    ie = import_reference(args.ref)
    sys.path.insert(0, ROOT)
    import importlib.util
    spec = importlib.util.spec_from_file_location("ie_program", os.path.join(ROOT, "interpolation-engine_amd", "program.py"))
    prog = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(prog)
    sys.modules["json5"].loads = prog.loads
    ie.json5 = sys.modules["json5"]
    with tempfile.TemporaryDirectory() as d:
        for rel, text in FILES.items():
            os.makedirs(os.path.dirname(os.path.join(d, rel)), exist_ok=True)
            with open(os.path.join(d, rel), "w") as f:
                f.write(text)
        ie.inserts_dir = d
        cases = []
        for s in CASES:
            rec = classify(ie, dict(INSERTS), s)
            if s == "{HH:MM}":
                continue  # the clock: covered by the main fixtures
            rec["s"] = s
            cases.append(rec)
    with tempfile.TemporaryDirectory() as base:
        d = os.path.join(base, "dir")
        for rel, text in FILES.items():
            os.makedirs(os.path.dirname(os.path.join(d, rel)), exist_ok=True)
            with open(os.path.join(d, rel), "w") as f:
                f.write(text)
        for rel, text in OUTSIDE_FILES.items():
            os.makedirs(os.path.dirname(os.path.join(base, rel)), exist_ok=True)
            with open(os.path.join(base, rel), "w") as f:
                f.write(text)
        for rel, hx in BAD_FILES.items():
            with open(os.path.join(d, rel), "wb") as f:
                f.write(bytes.fromhex(hx))
        ie.inserts_dir = d
        outside = []
        for s in OUTSIDE_CASES:
            rec = classify(ie, dict(INSERTS, **OUTSIDE_INSERTS), s, other_errors=True)
            rec["s"] = s
            outside.append(rec)
    with open(os.path.join(HERE, "inserts_dir_py.json"), "w", encoding="utf-8") as f:
        json.dump({"files": FILES, "inserts": INSERTS, "cases": cases, "outside_files": OUTSIDE_FILES,
                   "bad_files": BAD_FILES, "outside_inserts": OUTSIDE_INSERTS, "outside_cases": outside}, f,
                  ensure_ascii=False, indent=0)
    print("inserts_dir_py.json: %d cases, %d outside / bad-file cases" % (len(cases), len(outside)))


if __name__ == "__main__":
    main()
