"""set_interpdata on a built table set (ie_table_set_update; py:470-471, the stores of py:1566-1568
and 1770-1773 that the reference's loop makes between two interpolations): states are mutated
between two batches (values rewritten, keys added, including 17-32 byte keys, keys deleted,
brace-bearing values, typed values), the device copy is updated in place, and every string of the
second batch is compared with the oracle resolving it against its state's mutated dict. Also: the
pre-resolved values of a changed state go back to raw (they were resolved against the old dict),
and the clock entries follow their slots when a new key re-places their pilot group."""
import random

import pytest

import __graft_entry__ as G
from oracle import oracle as O

pytestmark = pytest.mark.gpu

G.build()
PKG = G.load_package()
IE = PKG.interpolation_engine
N = PKG._native
CLOCK = (12, 34, 56)


def _check(tset, states, strings, ids):
    got = tset.run(strings, ids)
    refs = [O.Oracle(d, "py", clock=tset.clock) for d in states]
    bad = []
    for s, t, (st, payload) in zip(strings, ids, got):
        rst, rout, rvid = refs[t].interpolate(s)
        name = N.STATUS_NAMES[st]
        want_value = refs[t].values[rvid] if rst == "OK_VALUE" and rvid < len(refs[t].values) else None
        if name != rst or (rst == "OK_STR" and payload != rout) or (rst == "OK_VALUE" and tset.value(payload) != want_value):
            bad.append((t, s, name, payload, rst, rout))
    return bad


def _strings(rng, states, per_state):
    strings, ids = [], []
    for t, d in enumerate(states):
        keys = list(d) + ["missing", "new-%d" % t, "long-key-%d-abcdefghijklmnop" % t]
        for _ in range(per_state):
            k = rng.choice(keys)
            form = rng.randrange(5)
            s = ("x{%s}y" % k, "{%s}" % k, "{q-{i%d}}!" % rng.randrange(4), "a{%s}b{%s}" % (k, rng.choice(keys)),
                 "plain %d" % t)[form]
            strings.append(s)
            ids.append(t)
    return strings, ids


def test_updates_match_the_oracle_on_mutated_states():
    rng = random.Random(11)
    states = []
    for t in range(300):
        d = {"name": "n%d" % t, "i%d" % (t % 4): t % 7, "q-%d" % (t % 7): "Q%d" % t, "count": t,
             "tmpl": "{name}!" if t % 3 == 0 else "static", "lst": ["a", t]}
        for j in range(t % 5):
            d["k%d" % j] = "v%d-%d" % (t, j)
        states.append(d)
    tset = IE.InsertsTableSet(states, clock=CLOCK)
    try:
        strings, ids = _strings(rng, states, 12)
        assert not _check(tset, states, strings, ids)
        # mutate: rewrite, add (short and 17-32 byte keys), delete, brace-bearing and typed values
        changes = []
        for t, d in enumerate(states):
            ops = [("name", "N%d" % t), ("new-%d" % t, "fresh%d" % t),
                   ("long-key-%d-abcdefghijklmnop" % t, "L%d" % t), ("tmpl", "{name}?{count}"),
                   ("count", t * 10), ("lst", ["b", t, "{x}"]), ("k0", IE.DELETE)]
            for k, v in rng.sample(ops, 4):
                if v is IE.DELETE:
                    if k in d:
                        del d[k]
                        changes.append((t, k, v))
                    continue
                d[k] = v
                changes.append((t, k, v))
        assert tset.update(changes)
        strings, ids = _strings(rng, states, 12)
        bad = _check(tset, states, strings, ids)
        assert not bad, (len(bad), bad[:6])
        # and a second round of updates on the updated table set
        changes = [(t, "name", "again%d" % t) for t in range(0, 300, 3)]
        for t, k, v in changes:
            states[t][k] = v
        assert tset.update(changes)
        bad = _check(tset, states, strings, ids)
        assert not bad, (len(bad), bad[:6])
    finally:
        tset.close()


def test_preresolved_values_go_raw_when_their_state_changes():
    # 'a' holds braces: pre-resolved at build against b = 'B'; after b changes the device must not
    # keep the old resolution
    states = [{"a": "<{b}>", "b": "B"}, {"a": "<{b}>", "b": "C"}]
    tset = IE.InsertsTableSet(states, clock=CLOCK)
    try:
        assert [r for r in tset.results(["x{a}", "x{a}"], [0, 1])] == ["x<B>", "x<C>"]
        states[0]["b"] = "Z"
        assert tset.update([(0, "b", "Z")])
        assert tset.results(["x{a}", "x{a}", "{a}"], [0, 1, 0]) == ["x<Z>", "x<C>", "<{b}>"]
    finally:
        tset.close()


def test_clock_entries_follow_replaced_groups():
    # many new keys re-place pilot groups (some holding a clock entry); set_clock must still find
    # every table's clock entries
    states = [{"k": "v"} for _ in range(64)]
    tset = IE.InsertsTableSet(states, clock=CLOCK)
    try:
        # within the headroom IE_TABLE_MUTABLE leaves (slots for twice the built keys)
        changes = [(t, "new%d_%d" % (t, j), "x") for t in range(64) for j in range(2)]
        for t, k, v in changes:
            states[t][k] = v
        assert tset.update(changes)
        assert tset.set_clock((1, 2, 3))
        got = tset.results(["{HH:MM}|{HH:MM:SS}|{new%d_1}" % t for t in range(64)], list(range(64)))
        assert got == ["01:02|01:02:03|x"] * 64
    finally:
        tset.close()


def test_updates_beyond_the_headroom_ask_for_a_rebuild():
    # more new keys than the table set has free slots: update says so (False), and a rebuilt table
    # set answers for the grown dicts
    states = [{"k": "v"} for _ in range(64)]
    tset = IE.InsertsTableSet(states, clock=CLOCK)
    try:
        changes = [(t, "new%d_%d" % (t, j), "x") for t in range(64) for j in range(8)]
        for t, k, v in changes:
            states[t][k] = v
        assert not tset.update(changes)
    finally:
        tset.close()
    tset = IE.InsertsTableSet(states, clock=CLOCK)
    try:
        got = tset.results(["{k}{new%d_7}" % t for t in range(64)], list(range(64)))
        assert got == ["vx"] * 64
    finally:
        tset.close()
