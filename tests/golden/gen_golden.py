#!/usr/bin/env python3
"""Generate golden vectors for the `{key}` hot path from the REFERENCE Python implementation.

Runs only in the build container, where /root/reference exists (it never travels to the GPU
box). The reference module is imported *by path at run time* with its three absent,
hot-path-irrelevant third-party imports (json5, openai, prompt_toolkit) stubbed in
sys.modules; nothing from the reference is copied into this repository — only the
input/output vectors it produces are written, as JSON data:

  tables.json           the insert dicts the cases run against (JSON values keep their types)
  interp_py.jsonl       interpolate_inserts(inserts, s)           py:497-541
  escape_py.jsonl       recursive_escape / recursive_unescape(s)  py:1436-1460
  simple_py.jsonl       get_simple_insertkey(s)                   py:477-495

Clock keys ('HH:MM', 'HH:MM:SS', py:433-436) are pinned by replacing the module's `datetime`
with a fixed clock (12:34:56). Cases that do not terminate within CASE_TIMEOUT seconds (the
reference loops forever on self-referential values) are recorded with status "DIVERGED".

Usage:  python tests/golden/gen_golden.py [--ref /root/reference/src]
"""
import argparse
import json
import os
import random
import signal
import sys
import types

HERE = os.path.dirname(os.path.abspath(__file__))
CASE_TIMEOUT = 0.25
CLOCK = (12, 34, 56)


def import_reference(src):
    for name in ["json5", "openai", "prompt_toolkit", "prompt_toolkit.application",
                 "prompt_toolkit.filters", "prompt_toolkit.history", "prompt_toolkit.key_binding",
                 "prompt_toolkit.layout", "prompt_toolkit.buffer", "prompt_toolkit.document",
                 "prompt_toolkit.layout.dimension", "prompt_toolkit.layout.controls",
                 "prompt_toolkit.styles", "prompt_toolkit.widgets", "prompt_toolkit.data_structures"]:
        m = types.ModuleType(name)
        m.__getattr__ = lambda attr: type(attr, (), {"from_dict": staticmethod(lambda *a, **k: None)})
        sys.modules[name] = m
    sys.path.insert(0, src)
    from interpolation_engine import interpolation_engine as ie  # noqa: E402

    class _FixedNow:
        def strftime(self, fmt):
            h, m, s = CLOCK
            return fmt.replace("%H", "%02d" % h).replace("%M", "%02d" % m).replace("%S", "%02d" % s)

    class _FixedDateTime:
        @staticmethod
        def now():
            return _FixedNow()

    ie.datetime = _FixedDateTime
    return ie


class _Timeout(Exception):
    pass


def _alarm(signum, frame):
    raise _Timeout()


def fnv1a(text):
    h = 0xCBF29CE484222325
    for b in text.encode("utf-8", "surrogatepass"):
        h = ((h ^ b) * 0x100000001B3) & 0xFFFFFFFFFFFFFFFF
    return h


def classify(ie, inserts, s):
    """Run the reference on one string; return a JSON-able record of its outcome."""
    protected = s.replace("\\{", ".〠").replace("\\}", "〠.")
    simple = bool(ie.get_simple_insertkey(protected))
    signal.signal(signal.SIGALRM, _alarm)
    signal.setitimer(signal.ITIMER_REAL, CASE_TIMEOUT)
    try:
        r = ie.interpolate_inserts(inserts, s)
    except _Timeout:
        return {"st": "DIVERGED"}
    except ie.InterpolationException as e:
        # the message names the failed lookup's key and lists the table's keys (py:430-467): its
        # first 96 characters and an FNV-1a of the whole
        return {"st": "E_INTERP", "msg_head": str(e)[:96], "msg_fnv": fnv1a(str(e))}
    except AssertionError as e:
        msg = str(e)
        if "trying to interpolate variable" in msg:
            return {"st": "E_ASSERT_TYPE"}
        return {"st": "E_ASSERT_BRACES"}
    except TypeError as e:
        if "unhashable" in str(e):
            return {"st": "E_UNHASHABLE"}
        raise
    except (RecursionError, MemoryError):
        return {"st": "DIVERGED"}
    finally:
        signal.setitimer(signal.ITIMER_REAL, 0)
    if simple:
        keys = [k for k, v in inserts.items() if v is r]
        rec = {"st": "OK_VALUE", "vkeys": keys}
        if not keys:
            # a fresh object: only the clock keys produce one
            h, m, sec = CLOCK
            if r == "%02d:%02d" % (h, m):
                rec["vkeys"] = ["@HH:MM"]
            elif r == "%02d:%02d:%02d" % (h, m, sec):
                rec["vkeys"] = ["@HH:MM:SS"]
            else:
                raise RuntimeError("typed result with no identity: %r -> %r" % (s, r))
        return rec
    assert isinstance(r, str), (s, r)
    return {"st": "OK_STR", "out": r}


# ---------------------------------------------------------------------------------------------
# tables
# ---------------------------------------------------------------------------------------------

def named_table():
    return {
        "name": "tom", "question-3": "Why?", "i": 3, "a": "{b}", "b": "B", "L": ["x", "y"],
        "n": 5, "big": 12345678901234567890123, "neg": -5, "z": 0, "bs": "q\\", "open": "}{",
        "k": "K", "x-B": "XB", "f": 1.5, "t": True, "d": {"k": 1}, "none": None,
        "q-1": "{b}-{b}", "q-3": "three", "d-D": "DEEP", "c-DEEP": "D2", "b-D2": "D3",
        "a-D3": "DEEP", "u": "ü€😀", "nl": "l1\nl2", "e": "", "uni": "héllo〠", "lb": "{",
        "rb": "}", "HH:MM": "shadowed", "ARG1": "first", "dot": "end.", "esc": "\\{x\\}",
        "bsb": "\\", "cl": "\\}", "ph": ".〠", "ph2": "〠.", "LL": [["a"], 2, "c\\"],
        "empty_list": [], "ints": [1, 2], "key with space": "spaced", "é": "accent",
        "{b}": "braced-key", "5": "five", "B": "bee", "K": "kay", "Why?": "because",
        "tom": "{name}", "loop": "{loop}", "grow": "{grow}{grow}", "aa": "{b}{b}",
        "nest": "{a}", "self": "x{self}", "\\{x\\}": "escaped-key", "x\\{": "xesc",
        "}n{": "NEGKEY", "}{": "braces-key",
    }


def named_cases():
    c = [
        "My name is {name}.", "{question-{i}}", "{a}", "x{a}y", "{q-{i}}", "x{q-{i}}",
        "{q-1}", "x{q-1}", "{a-{b-{c-{d}}}}", "x{a-{b-{c-{d}}}}y", "{d-D}", "{c-{d-D}}",
        "{L}", "x{L}y", "{n}", "n={n}", "n={big}", "n={neg}{z}", "x{f}", "x{t}", "x{d}",
        "x{none}", "{f}", "{d}", "{none}", "{t}", "{}", "x{}", "{{}}", "a{b", "{{k}", "{lb}x}",
        "a}b", "}{", "{k}{open}", "{{a}}", "{{n}}", "{{L}}", "{{d}}", "{{f}}", "{{none}}",
        "{{t}}", "{x{bs}}", "y{x{bs}}", "\\{name\\} {name}", "a\\{b\\}c{k}", "{k}\\}",
        "\\{{k}\\}", "\\\\{k}", "x.〠y", "{uni}x", "<{u}>", "{nl}", "[{e}]", "{HH:MM}",
        "{HH:MM:SS}", "at {HH:MM}", "at {HH:MM:SS}!", "{ARG1}", "{ARG2}", "x{ARG1}",
        "{ARG}", "x{ARG}", "{dot}\\}", "x{dot}\\}", "\\}\\}", ".\\}", "a.\\}b", "{esc}",
        "x{esc}", "{{esc}}", "x{bsb}", "x{bsb}y", "{bsb}{k}", "x{bsb}{k}", "{cl}", "x{cl}",
        ".{cl}", "x.{cl}", "{ph}", "x{ph}", "x{ph2}", "{LL}", "x{LL}", "x{empty_list}",
        "x{ints}", "{key with space}", "x{é}", "{{b}}", "{\\{b\\}}", "x{\\{x\\}}", "{x\\{}",
        "x{x\\{}y", "{{k}}", "{K}", "{{name}}", "x{tom}", "{tom}", "{nest}", "x{nest}",
        "x{aa}", "{aa}", "x{loop}", "x{grow}", "{self}", "x{self}", "", "plain", "{",
        "}", "\\", "\\{", "\\}", "{\\}", "{k\\}", "{k}}", "{{k}}}", "}{k}{", "{k}}{",
        "a{k}b{k}c", "{k}{k}", "{k}-{n}", "{{k}-{n}}", "x{5}", "{5}", "{{5}}", "{{{i}}}",
        "{question-{{i}}}", "x{question-{i}}y", "{missing}", "x{missing}", "x{missing}{f}",
        "x{f}{missing}", "{missing}{k}", "x{a{missing}}", "x{k}{missing-{f}}", "x{{f}}",
        "x{ {k} }", "{ k}", "x{n}{L}{k}", "x{{L}}", "{x}{", "\\{}", "{\\{}", "{}}", "{{}",
        "x\\\\{k}", "x\\\\\\{k}", "\\\\\\\\", "é{k}é", "😀{u}😀", "{k}\n{k}", "〠", ".〠",
        "〠.", "{k}.〠", "〠.{k}", "x{k}〠y", "a.\\{b", "a\\}.b", "\\{.\\}", "\\}.\\{",
        "x{dot}{cl}", "{dot}{cl}", "x{k}\\}\\}", "x\\}{k}", "{k}{bsb}", "{bsb}",
        # get_simple_insertkey has no brace test at the edges (py:485-495): the depth may dip below
        # 0 and come back at the last character, so these are whole-string forms too
        "a}n{b", "a}b{c", "k}{\\", "é}n{é", "😀}n{😀", "a}{b", "x}{y}{z", "a}n{", "}n{b", "a}}n{{b",
        "a}{k}{b", "é}{é", "a}n{{k}", "a}\\{n{b",
    ]
    return c


KEY_ALPH = ["a", "b", "c", "ab", "k", "x-", "-", ".", "\\", "é", " ", "0", "1"]
VAL_TOKENS = ["a", "b", "c", "x", "y", "ab", " ", ".", "-", "é", "€", "😀", "\n", "\\", "{", "}",
              "\\{", "\\}", "〠", ".〠", "〠.", "{a}", "{b}", "{ab}", "{k}", "0", "9"]


def rand_key(rng):
    n = rng.choice([1, 1, 1, 2, 2, 3])
    return "".join(rng.choice(KEY_ALPH) for _ in range(n))


def rand_value(rng, keys):
    r = rng.random()
    if r < 0.55:
        n = rng.randint(0, 6)
        toks = []
        for _ in range(n):
            if rng.random() < 0.7:
                toks.append(rng.choice(["a", "b", "c", "x", "y", "z", "ab", " ", "-", "0", "é"]))
            else:
                toks.append(rng.choice(VAL_TOKENS + ["{%s}" % rng.choice(keys)]))
        return "".join(toks)
    if r < 0.68:
        return rng.choice([0, 1, 7, -3, 42, 99999999999999999999, rng.randint(-1000, 1000)])
    if r < 0.76:
        return [rng.choice(["a", "b", 1, "c\\", "{a}"]) for _ in range(rng.randint(0, 3))]
    if r < 0.82:
        return rng.choice([1.5, -0.25, 2.0])
    if r < 0.88:
        return rng.choice([True, False])
    if r < 0.93:
        return None
    return {"k": rng.randint(0, 3)}


def random_table(rng, n_keys):
    keys = []
    while len(keys) < n_keys:
        k = rand_key(rng)
        if k not in keys:
            keys.append(k)
    t = {}
    for k in keys:
        t[k] = rand_value(rng, keys)
    if rng.random() < 0.5:
        t["HH:MM"] = "shadow"
    return t


TPL_TOKENS = ["a", "b", "x", " ", ".", "-", "é", "😀", "\n", "\\", "{", "}", "\\{", "\\}",
              "〠", ".〠", "〠.", "\\\\"]


def rand_ref(rng, keys, depth):
    """A properly nested reference, possibly with nested refs inside its key."""
    if depth > 0 and rng.random() < 0.35:
        k = rng.choice(keys)
        cut = rng.randint(0, len(k))
        return "{" + k[:cut] + rand_ref(rng, keys, depth - 1) + k[cut:] + "}"
    if rng.random() < 0.85:
        return "{" + rng.choice(keys) + "}"
    return "{" + rand_key(rng) + "}"


def rand_template(rng, keys, mode):
    toks = []
    n = rng.randint(0, 7)
    for _ in range(n):
        r = rng.random()
        if mode == "structured":
            if r < 0.45:
                toks.append(rng.choice(["a", "b", "x", " ", "-", "é", "😀", ".", "tt"]))
            elif r < 0.8:
                toks.append(rand_ref(rng, keys, 3))
            else:
                toks.append(rng.choice(["\\{", "\\}", "\\{lit\\}", "\\\\", "\\"]))
        else:
            if r < 0.3:
                toks.append(rand_ref(rng, keys, 2))
            else:
                toks.append(rng.choice(TPL_TOKENS))
    s = "".join(toks)
    if mode == "structured" and rng.random() < 0.2:
        s = rand_ref(rng, keys, 3)  # whole-string simple form
    return s


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference/src")
    ap.add_argument("--seed", type=int, default=20261015)
    ap.add_argument("--random-tables", type=int, default=6)
    ap.add_argument("--cases-per-table", type=int, default=900)
    args = ap.parse_args()

    ie = import_reference(args.ref)
    rng = random.Random(args.seed)

    tables = [named_table()]
    for _ in range(args.random_tables):
        tables.append(random_table(rng, rng.randint(4, 14)))
    # a table of only inert values (the fast path's home ground)
    inert = {"k%d" % j: "v%d%s" % (j, rng.choice(["", "é", " x", "-y", "\\{e\\}"])) for j in range(30)}
    inert.update({"q-%d" % j: "Q%d" % j for j in range(20)})
    inert.update({"i%d" % j: j % 20 for j in range(10)})
    tables.append(inert)

    rows = []
    for s in named_cases():
        rows.append(dict({"t": 0, "s": s, "tag": "named"}, **classify(ie, tables[0], s)))
    for ti in range(1, len(tables)):
        keys = list(tables[ti].keys())
        for j in range(args.cases_per_table):
            mode = "structured" if j % 2 == 0 else "chaotic"
            s = rand_template(rng, keys, mode)
            rows.append(dict({"t": ti, "s": s, "tag": mode}, **classify(ie, tables[ti], s)))
    # inert table: config-3-like nested refs with filler and escapes
    ti = len(tables) - 1
    for j in range(600):
        parts = []
        for _ in range(rng.randint(1, 4)):
            parts.append(rng.choice(["ab", "é ", "x.", "😀", "\\{lit\\}", "-", "z"]))
            parts.append(rng.choice(["{k%d}" % rng.randrange(30), "{q-{i%d}}" % rng.randrange(10),
                                     "{k%d}" % rng.randrange(40)]))
        rows.append(dict({"t": ti, "s": "".join(parts), "tag": "inert"}, **classify(ie, tables[ti], "".join(parts))))

    with open(os.path.join(HERE, "tables.json"), "w", encoding="utf-8") as f:
        json.dump(tables, f, ensure_ascii=False, indent=0)
    with open(os.path.join(HERE, "interp_py.jsonl"), "w", encoding="utf-8") as f:
        for r in rows:
            f.write(json.dumps(r, ensure_ascii=False) + "\n")

    esc_inputs = ["", "a", "{", "}", "\\{", "\\}", "\\\\{", "{a}", "\\{a\\}", "a{b}c\\{", "a\\{b\\}c\\\\{d",
                  "}{", "{{}}", "\\\\\\", "é{😀}", ".〠", "〠.", "\\{\\}\\{", "x\\y\\{"]
    for _ in range(400):
        esc_inputs.append("".join(rng.choice(TPL_TOKENS) for _ in range(rng.randint(0, 10))))
    with open(os.path.join(HERE, "escape_py.jsonl"), "w", encoding="utf-8") as f:
        for s in esc_inputs:
            f.write(json.dumps({"s": s, "esc": ie.recursive_escape(s), "unesc": ie.recursive_unescape(s)},
                               ensure_ascii=False) + "\n")

    simple_inputs = ["{a}", "{{a}/b}", "{a}/{b}", "ab", "a", "", "{}", "{a}}", "}a{", "{{}}", "{é}",
                     "é", "{a}{b}", "{{a}{b}}", "{", "}", "x{a}", "{a}x", "{{{a}}}", "{\n}"]
    for _ in range(300):
        simple_inputs.append("".join(rng.choice(["{", "}", "a", "é", "{a}", "."]) for _ in range(rng.randint(0, 8))))
    with open(os.path.join(HERE, "simple_py.jsonl"), "w", encoding="utf-8") as f:
        for s in simple_inputs:
            f.write(json.dumps({"s": s, "key": ie.get_simple_insertkey(s)}, ensure_ascii=False) + "\n")
        f.write(json.dumps({"s": 5, "key": ie.get_simple_insertkey(5)}) + "\n")

    # recursive_interpolate over task-shaped structures (py:1462-1494)
    rtable = {"name": "tom", "i": 3, "question-3": "Why?", "persona_name": "Ann", "t1": {"cmd": "print", "text": "{name}"},
              "lst": ["{name}", "x{i}", 5], "a": "{b}", "b": "B", "tasks_ref": [{"cmd": "print", "text": "hi"}],
              "n": 7, "d": {"k": "{name}"}, "esc": "\\{raw\\}"}
    structs = [
        {"cmd": "print", "text": "My name is {name}."},
        {"cmd": "user_input", "prompt": "{question-{i}}", "output_name": "{persona_name}/answer-{i}"},
        {"cmd": "serial", "tasks": ["{t1}", {"cmd": "print", "text": "{undefined_later}"}]},
        {"cmd": "for", "tasks": "{tasks_ref}", "x": "{name}"},
        {"cmd": "goto_map", "value": "{missing}", "map": {"a": 1}},
        {"cmd": "replace_map", "item": "{missing}"},
        {"cmd": "set", "item": "{lst}", "output_name": "out-{i}"},
        {"cmd": "set", "item": "{a}", "output_name": "o"},
        {"cmd": "set", "item": "{d}", "output_name": "o"},
        {"cmd": "set", "item": ["{name}", ["{i}", "{n}x"], {"{name}": "{i}"}], "output_name": "o"},
        {"cmd": "print", "text": "{esc} and \\{name\\}"},
        {"cmd": "print", "text": "{missing}"},
        {"cmd": "print", "text": "a{b"},
        ["{name}", "{i}", 3, None, True, 1.5],
        "{lst}",
        "{i}",
        5,
    ]
    with open(os.path.join(HERE, "recursive_py.jsonl"), "w", encoding="utf-8") as f:
        f.write(json.dumps({"table": rtable}, ensure_ascii=False) + "\n")
        for x in structs:
            try:
                r = ie.recursive_interpolate(rtable, x)
                rec = {"x": x, "st": "OK", "out": r}
            except ie.InterpolationException:
                rec = {"x": x, "st": "E_INTERP"}
            except AssertionError:
                rec = {"x": x, "st": "ASSERT"}
            f.write(json.dumps(rec, ensure_ascii=False) + "\n")
        for x in structs:
            f.write(json.dumps({"esc_in": x, "esc": ie.recursive_escape(x), "unesc": ie.recursive_unescape(x)},
                               ensure_ascii=False) + "\n")

    from collections import Counter
    print("interp rows:", len(rows), Counter(r["st"] for r in rows))


if __name__ == "__main__":
    main()
