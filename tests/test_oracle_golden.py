"""Pin the C oracle against the reference's own outputs (tests/golden/, made by gen_golden.py).

CPU only. The oracle is the checker for every GPU parity test, so it must reproduce every
golden vector exactly: byte-identical strings, identical status class, identical typed value.
"""
import pytest

from oracle import oracle as O
from tests.conftest import load_golden

VID_SPECIAL = {"@HH:MM": O.VID_HHMM, "@HH:MM:SS": O.VID_HHMMSS}


def _expected_vids(row, keys):
    out = set()
    for k in row["vkeys"]:
        out.add(VID_SPECIAL[k] if k in VID_SPECIAL else keys.index(k))
    return out


def test_oracle_matches_reference_golden(golden_tables, golden_interp):
    oracles = [O.Oracle(t, "py") for t in golden_tables]
    bad = []
    for row in golden_interp:
        o = oracles[row["t"]]
        st, out, vid = o.interpolate(row["s"])
        ok = st == row["st"]
        if ok and st == "OK_STR":
            ok = out == row["out"]
        if ok and st == "OK_VALUE":
            ok = vid in _expected_vids(row, o.keys)
        if not ok:
            bad.append((row, st, out, vid))
    assert not bad, "%d mismatches, first: %r" % (len(bad), bad[:5])


def test_golden_covers_every_status(golden_interp):
    seen = {r["st"] for r in golden_interp}
    for st in ["OK_STR", "OK_VALUE", "E_INTERP", "E_ASSERT_BRACES", "E_ASSERT_TYPE", "E_UNHASHABLE", "DIVERGED"]:
        assert st in seen, st


def test_oracle_escape_golden():
    for row in load_golden("escape_py.jsonl"):
        assert O.escape(row["s"]) == row["esc"], row
        assert O.escape(row["s"], unescape=True) == row["unesc"], row


def test_oracle_simple_insertkey_golden():
    for row in load_golden("simple_py.jsonl"):
        if not isinstance(row["s"], str):
            continue  # non-str input: the reference returns None (py:481-482); callers only pass str
        got = O.simple_insertkey(row["s"], "py")
        want = row["key"]
        # py returns '' (falsy) or None for "not simple"; the C API reports truthiness
        assert (got or None) == (want or None), row


@pytest.mark.parametrize("s,want", [
    ("{a}", ("OK_VALUE", None)),
    ("x{L}y", ("OK_STR", "xxyy")),          # D1: rs joins lists
    ("x{f}", ("OK_STR", "x1.5")),           # D2: rs splices floats
    ("{k}{open}", ("E_RS_PANIC", None)),    # D3: rs unwrap() panics on the '}{' leftover
    ("{{n}}", ("OK_VALUE", None)),          # D4: rs value_to_string(5) == "5" is a key here
    ("x{t}", ("E_ASSERT_TYPE", None)),      # bool is not splicable in rs either
    ("{}", ("E_INTERP", None)),             # D10
    # derived line by line from interp.rs:31-89 (interpolate_inserts), 91-137 (get_interpdata),
    # 314-322 (value_to_string)
    ("x{nested}y", ("E_INTERP", None)),     # :74 join -> 'p12{"z":1}'; the loop (:55) re-reads '{"z":1}' as a key
    ("x{none}y", ("E_ASSERT_TYPE", None)),  # :76-79 Null is unsupported
    ("x{obj}y", ("E_ASSERT_TYPE", None)),   # :76-79 Object is unsupported
    ("x{n}y", ("OK_STR", "x5y")),           # :73 Number::to_string
    ("x{neg}y", ("OK_STR", "x-3y")),
    ("x{two}", ("OK_STR", "x2.0")),         # serde_json prints f64 2.0 as "2.0"
    ("{q-{i}}", ("OK_VALUE", "q-5")),       # :50-51 the key is interpolated first: "q-5"
    ("a{e}b", ("OK_STR", "ab")),
    ("\\{a\\}", ("OK_STR", "\\{a\\}")),    # :42-43 protected, :84-85 restored
    ("{a", ("E_ASSERT_BRACES", None)),      # :56-61 uneven count
    ("a}", ("OK_STR", "a}")),               # :54 no '{': the loop never runs
    ("{bs}x", ("OK_STR", "q\\x")),
    ("{bs}{a}", ("OK_STR", "q\\A")),        # rightmost first: {a}, then {bs}
    ("{a}{bs}", ("OK_STR", "Aq\\")),
    ("{t}", ("OK_VALUE", "t")),             # :44-52 simple path returns the Bool itself
    ("{{a}}", ("E_INTERP", None)),          # :46-48 subkey a -> "A" is then the key: missing
    ("{{f}}", ("E_INTERP", None)),          # value_to_string(1.5) = "1.5": missing
    ("{5}", ("OK_VALUE", "5")),
    ("x{}y", ("E_INTERP", None)),           # :103 '' key
    ("{ARG1}", ("E_INTERP", None)),         # :109-115 ARGn not provided
    ("}{", ("E_RS_PANIC", None)),           # :63-66 no '}' after the last '{': unwrap() on None
    ("a}{b", ("E_RS_PANIC", None)),
    ("x{L}{L}", ("OK_STR", "xxyxy")),
    ("n={big}", ("OK_STR", "n=12345678901234567890")),
])
def test_oracle_rust_dialect_restated(s, want):
    """Rust dialect: hand-derived from rust-project/src/interp.rs (parity unpinned).
    For OK_VALUE the second field names the key whose value is returned."""
    t = {"a": "A", "L": ["x", "y"], "f": 1.5, "k": "K", "open": "}{", "n": 5, "5": "five", "t": True,
         "nested": ["p", [1, 2], {"z": 1}], "none": None, "obj": {"b": 2}, "q-5": "Q5", "i": 5, "neg": -3,
         "two": 2.0, "bs": "q\\", "e": "", "big": 12345678901234567890}
    o = O.Oracle(t, "rs")
    st, out, vid = o.interpolate(s)
    assert st == want[0]
    if want[1] is not None and st == "OK_STR":
        assert out == want[1]
    if want[1] is not None and st == "OK_VALUE":
        assert list(t)[vid] == want[1]


def _unescape_cmd_oracle(table, strings):
    """The oracle's unescape command (ieo_run_batch mode 1) over strings -> (statuses, hashes, vids)."""
    import numpy as np
    o = O.Oracle(table, "py")
    bs = [O.enc(s) for s in strings]
    offs = np.zeros(len(bs) + 1, np.uint64)
    offs[1:] = np.cumsum([len(b) for b in bs])
    blob = np.frombuffer(b"".join(bs) + b"\0", np.uint8)
    n = len(bs)
    st, ln, hs, vid = np.zeros(n, np.uint8), np.zeros(n, np.uint64), np.zeros(n, np.uint64), np.zeros(n, np.uint32)
    o.run_batch(blob, offs, n, 4, st, ln, hs, vid, command_only=True)
    return o, [O.STATUS_NAMES[k] for k in st], hs, vid


def test_oracle_unescape_command_matches_reference():
    """The `unescape` command (py:1660-1667) on the reference-generated vectors: the oracle gives
    the reference's result wherever recursive_interpolate does not re-enter a whole-string result;
    where it does (py:1463-1464), it reports RECURSE, which must be exactly the items that are a
    whole-string '{key}' after the unescape and whose interpolation is a str, list or dict."""
    g = load_golden("unescape_cmd_py.json")
    table, rows = g["table"], g["rows"]
    o, st, hs, vid = _unescape_cmd_oracle(table, [r["s"] for r in rows])
    keys = list(table.keys())
    bad, n_rec = [], 0
    for k, r in enumerate(rows):
        u = r["s"].replace("\\{", "{").replace("\\}", "}")
        simple = bool(O.simple_insertkey(u)) and len(u) >= 3
        if st[k] == "RECURSE":
            n_rec += 1
            if not simple:
                bad.append(("recurse on a non-simple item", r, st[k]))
            continue
        if st[k] != r["st"]:
            bad.append((r, st[k]))
        elif st[k] == "OK_STR" and int(hs[k]) != O.fnv1a(O.enc(r["out"])):
            bad.append((r, "bytes"))
        elif st[k] == "OK_VALUE":
            v = table[keys[vid[k]]] if vid[k] < len(keys) else None
            if simple and isinstance(v, (str, list, dict)):
                bad.append(("typed container result not re-entered", r))
            elif v != r["value"] and vid[k] < len(keys):
                bad.append((r, "value", v))
    assert not bad, (len(bad), bad[:5])
    assert n_rec > 20  # the fixture exercises the recursion
