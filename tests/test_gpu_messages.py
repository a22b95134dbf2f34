"""The reference's own exception text for strings whose lookup misses (py:430-467, get_interpdata's
messages: the missing key, the table's keys, the ARGn and empty-key forms) through the mirror:
the device records the failed lookup's key (IE_OPT_ERROR_KEYS, the literal path) and the mirror
writes the message from it. Compared with what the reference raised on the same strings
(tests/golden/gen_golden.py: msg_head + FNV-1a of the whole message)."""
import pytest

import __graft_entry__ as G

pytestmark = pytest.mark.gpu

G.build()
PKG = G.load_package()
CLOCK = (12, 34, 56)


def fnv1a(text):
    h = 0xCBF29CE484222325
    for b in text.encode("utf-8", "surrogatepass"):
        h = ((h ^ b) * 0x100000001B3) & 0xFFFFFFFFFFFFFFFF
    return h


def test_missing_key_messages_match_reference(golden_tables, golden_interp):
    by_t = {}
    for r in golden_interp:
        if r["st"] == "E_INTERP" and "msg_fnv" in r:
            by_t.setdefault(r["t"], []).append(r)
    bad, n = [], 0
    for ti, rows in sorted(by_t.items()):
        t = PKG.InsertsTable(golden_tables[ti], clock=CLOCK)
        try:
            got = t.results([r["s"] for r in rows])
        finally:
            t.close()
        for r, g in zip(rows, got):
            n += 1
            if not isinstance(g, PKG.InterpolationException) or fnv1a(str(g)) != r["msg_fnv"]:
                bad.append((ti, r["s"], r["msg_head"], str(g)[:120]))
    assert n > 1000
    assert not bad, (len(bad), bad[:5])


def test_single_string_message():
    with pytest.raises(PKG.InterpolationException) as e:
        PKG.interpolate_inserts({"name": "tom", "n": 5}, "Hi {q-{n}}!")
    assert str(e.value) == "Could not find variable 'q-5' in interpdata. Available interpolation data keys are ['name', 'n']."
    with pytest.raises(PKG.InterpolationException) as e:
        PKG.interpolate_inserts({"name": "tom"}, "x{ARG2}")
    assert str(e.value) == "Argument interpolation key 'ARG2' is used, but the user passed less than 2 program arguments."
