"""Host-side logic of the mirror that runs without a GPU: the inserts-directory key rules used by
the host completion of IE_NEEDS_HOST (interpolation_engine.py), and the reduced dict a map value is
interpolated against (maps.py, replace_map's `inserts | extra_inserts`, py:1736-1738)."""
import __graft_entry__ as G

G.load_package()
from interpolation_engine_amd import interpolation_engine as IE  # noqa: E402
from interpolation_engine_amd import maps as M  # noqa: E402


def test_canonical_key_matches_the_device_rule():
    """ie_device.h missing_status: components separated by single '/', none empty, '.' or '..',
    no NUL; '' is a plain miss (canonical)."""
    for k, want in [("x", True), ("sub/leaf", True), ("", True), ("a.b", True), ("..x", True),
                    ("../x", False), ("a//b", False), ("./x", False), ("x/", False), ("/abs", False),
                    ("..", False), ("a/./b", False), ("a\0b", False)]:
        assert IE._canonical_key(k) == want, k


def test_literal_keys_are_the_innermost_pairs():
    assert IE._literal_keys("a{b}c{d-{e}}") == ["b", "e"]
    assert IE._literal_keys("{../x} and {sub/../y}") == ["../x", "sub/../y"]
    assert IE._literal_keys("no pairs }{") == []


def test_value_dict_keeps_the_captures_and_what_the_value_reaches():
    state = {"a": "A", "b": "x{c}y", "c": "C", "d": "unused", "1": "shadowed", "n": 3, "L": ["{c}"]}
    caps = ["cap1", "cap2"]
    d = M._value_dict(state, "{1}-{a}-{b}", caps, "py")
    assert d == {"1": "cap1", "2": "cap2", "a": "A", "b": "x{c}y", "c": "C"}  # captures win over '1'
    # a list value renders with its braces, which the loop resolves again
    assert M._value_dict(state, "{L}", [], "py") == {"L": ["{c}"], "c": "C"}
    # a key built from another lookup cannot be known in advance: the whole state
    full = M._value_dict(state, "{q-{1}}", caps, "py")
    assert full == dict(state, **{"1": "cap1", "2": "cap2"})
    nested_value = dict(state, e="{q-{a}}")
    assert M._value_dict(nested_value, "{e}", [], "py") == nested_value
    # keys the state does not hold stay out (the device reports the miss, as the reference raises)
    assert M._value_dict(state, "{zz}", [], "py") == {}


def test_static_walk_is_the_state_walk_for_items_without_whole_string_keys():
    """replace_map_states walks an item once for all states when no node is a whole-string key
    (recursive_replace, py:1748-1759, then reads no state): the same skeleton and leaves as the
    per-state walk; an item with one raises, and the per-state walk runs."""
    state = {"a": "A", "k": "v{a}"}
    for item in ["plain", "x {a} y", ["{a} and {b}", "z", {"{a}-x": ["w", 3, None]}], {"k": {"n": 1.5}}, 7]:
        lv0, lv1 = [], []
        assert M._static_leaves(item, lv0) == M._leaves(state, item, lv1)
        assert lv0 == lv1
    for item in ["{a}", ["x", "{k}"], {"{a}": "y"}]:
        try:
            M._static_leaves(item, [])
        except M._StateDependent:
            continue
        raise AssertionError("%r holds a whole-string key" % (item,))
