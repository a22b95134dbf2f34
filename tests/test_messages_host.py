"""The host half of the reference's miss messages (no GPU): given the key a failed lookup used,
interpolation_engine._missing_key_exception writes get_interpdata's text (py:437-467) exactly. The
key is read back from the reference's own message head in the golden rows (gen_golden.py
msg_head), the message compared by FNV-1a with the reference's whole message."""
import re

import __graft_entry__ as G

PKG = G.load_package()
IE = PKG.interpolation_engine


def fnv1a(text):
    h = 0xCBF29CE484222325
    for b in text.encode("utf-8", "surrogatepass"):
        h = ((h ^ b) * 0x100000001B3) & 0xFFFFFFFFFFFFFFFF
    return h


def _key_of(head):
    m = re.match(r"Could not find variable '(.*)' in interpdata\. Available", head, re.S)
    if m:
        return m.group(1)
    m = re.match(r"Argument interpolation key '(.*)' is used, but", head, re.S)
    if m:
        return m.group(1)
    if head == "Tried to interpolate empty string ''.":
        return ""
    return None


def test_messages_from_the_missing_key(golden_tables, golden_interp):
    n = 0
    for r in golden_interp:
        if r["st"] != "E_INTERP" or "msg_fnv" not in r:
            continue
        key = _key_of(r["msg_head"])
        if key is None or len(r["msg_head"]) >= 96 and "' in interpdata" not in r["msg_head"]:
            continue  # a key too long for the recorded head
        e = IE._missing_key_exception(key, list(golden_tables[r["t"]].keys()), False)
        assert isinstance(e, IE.InterpolationException)
        assert fnv1a(str(e)) == r["msg_fnv"], (r["s"], r["msg_head"], str(e)[:120])
        n += 1
    assert n > 1000
