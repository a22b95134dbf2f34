"""set_interpdata on a built table set (ie_table_set_update; py:470-471, the stores of py:1566-1568
and 1770-1773 that the reference's loop makes between two interpolations): states are mutated
between two batches (values rewritten, keys added, including 17-32 byte keys, keys deleted,
brace-bearing values, typed values), the device copy is updated in place, and every string of the
second batch is compared with the oracle resolving it against its state's mutated dict. Also: the
pre-resolved values of a changed state go back to raw (they were resolved against the old dict),
the clock entries and pre-resolved values follow their slots when new keys re-place their pilot
groups, the text arena is compacted and stays bounded under config 5's rewrite pattern, and a
small forced arena limit gives IE_ERR_CAPACITY (a rebuild) instead of a wrapped offset."""
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
    tset = IE.InsertsTableSet(states, clock=CLOCK, mutable=True)
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
    tset = IE.InsertsTableSet(states, clock=CLOCK, mutable=True)
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
    tset = IE.InsertsTableSet(states, clock=CLOCK, mutable=True)
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
    tset = IE.InsertsTableSet(states, clock=CLOCK, mutable=True)
    try:
        changes = [(t, "new%d_%d" % (t, j), "x") for t in range(64) for j in range(8)]
        for t, k, v in changes:
            states[t][k] = v
        assert not tset.update(changes)
    finally:
        tset.close()
    tset = IE.InsertsTableSet(states, clock=CLOCK, mutable=True)
    try:
        got = tset.results(["{k}{new%d_7}" % t for t in range(64)], list(range(64)))
        assert got == ["vx"] * 64
    finally:
        tset.close()


def test_clock_and_preresolved_slots_survive_many_group_moves():
    # tables whose keys are mostly clock entries and pre-resolved values: every new key re-places its
    # pilot group, whose members often move into each other's old slots; after each round the clock
    # is re-set (every table's two clock entries must still be found) and a pre-resolved value's
    # dependency changes (its slot must still be listed, so that it goes back to raw)
    states = [{"a": "<{b}>", "b": "B%d" % t} for t in range(1500)]
    tset = IE.InsertsTableSet(states, clock=CLOCK, mutable=True)
    try:
        for rnd in range(2):
            changes = [(t, "n%d_%d" % (rnd, t), "x%d" % t) for t in range(len(states))]
            for t, k, v in changes:
                states[t][k] = v
            assert tset.update(changes)
            clk = (rnd + 1, 10 + rnd, 20 + rnd)
            assert tset.set_clock(clk)
            got = tset.results(["{HH:MM}|{HH:MM:SS}" for _ in states], list(range(len(states))))
            assert got == ["%02d:%02d|%02d:%02d:%02d" % (clk[0], clk[1], *clk)] * len(states)
        changes = [(t, "b", "Z%d" % t) for t in range(0, len(states), 2)]
        for t, k, v in changes:
            states[t][k] = v
        assert tset.update(changes)
        got = tset.results(["x{a}" for _ in states], list(range(len(states))))
        assert got == ["x<%s>" % st["b"] for st in states]
    finally:
        tset.close()


def test_arena_is_compacted_and_stays_bounded():
    # config 5's loop rewrites a long history text in every state every iteration: replaced texts
    # are counted dead and the arena is compacted once they outnumber the live bytes; every string
    # matches the oracle on the mutated states after every round
    rng = random.Random(5)
    states = [{"hist": "h%d" % t, "name": "n%d" % t, "short": "s"} for t in range(200)]
    tset = IE.InsertsTableSet(states, clock=CLOCK, mutable=True)
    try:
        for rnd in range(12):
            changes = []
            for t, d in enumerate(states):
                # growing histories (appended), and short rewrites that fit in place
                d["hist"] = d["hist"] + (" turn %d:%d " % (rnd, t)) * rng.randrange(1, 40)
                d["short"] = "s%d" % (rnd % 3)
                changes += [(t, "hist", d["hist"]), (t, "short", d["short"])]
            assert tset.update(changes)
            strings = ["{hist}|{short}|{name}" for _ in states] + ["x{short}y" for _ in states]
            bad = _check(tset, states, strings, list(range(len(states))) * 2)
            assert not bad, (rnd, bad[:3])
            size, live, comp = tset.arena_stats()
            # after every call the dead bytes are at most the live ones (or 64 KB)
            assert size <= 2 * live + (64 << 10) + 64, (rnd, size, live)
        size, live, comp = tset.arena_stats()
        assert comp >= 1, (size, live, comp)
        assert len(tset.values) <= sum(len(d) for d in states) + 2 * len(states)  # value ids reused
    finally:
        tset.close()


def test_arena_limit_reports_capacity_not_a_wrap():
    # a small forced limit: updates fit until the live texts exceed it, then update reports False
    # (IE_ERR_CAPACITY, rebuild) instead of wrapping an offset; what came before stays correct
    states = [{"v": "x", "w": "y"} for _ in range(64)]
    tset = IE.InsertsTableSet(states, clock=CLOCK, mutable=True)
    try:
        size0, live0, _ = tset.arena_stats()
        tset.set_arena_limit(size0 + 24 * 1024)
        ok_rounds = 0
        for rnd in range(40):
            changes = [(t, "v", "%d:" % rnd + "z" * (40 * rnd)) for t in range(64)]
            for t, k, v in changes:
                states[t][k] = v
            if not tset.update(changes):
                break
            ok_rounds += 1
            bad = _check(tset, states, ["{v}{w}" for _ in states], list(range(64)))
            assert not bad, (rnd, bad[:2])
        assert 0 < ok_rounds < 40
    finally:
        tset.close()
    tset = IE.InsertsTableSet(states, clock=CLOCK, mutable=True)
    try:
        assert not _check(tset, states, ["{v}{w}" for _ in states], list(range(64)))
    finally:
        tset.close()


def test_store_hands_out_value_ids():
    # ie_table_set_store: a rewrite keeps its key's id, a new key takes the next id (a set's build
    # gives kv i the id i), a delete frees its key's id and the next new key takes it; a typed
    # whole-string result names the id the store reported
    import ctypes
    states = [{"a": "x", "b": 1}, {"c": "y"}]
    tset = IE.InsertsTableSet(states, clock=CLOCK, mutable=True)
    P = N.pack_module()
    try:
        def store(changes):
            kv, tids, keep = P.pack(changes, len(states), IE.DELETE, IE.render, "py")
            out = (ctypes.c_uint32 * len(changes))()
            rc = N.lib().ie_table_set_store(tset.h, (ctypes.c_char * len(kv)).from_buffer(kv),
                                            (ctypes.c_char * len(tids)).from_buffer(tids), len(changes), out)
            assert rc == 0, N.STATUS_NAMES[rc] if rc < len(N.STATUS_NAMES) else rc
            return list(out)
        assert store([(0, "a", "x2"), (1, "d", 5), (0, "b", IE.DELETE), (1, "zz", IE.DELETE), (0, "", "e")]) == \
            [0, 3, 1, 0xFFFFFFFF, 0xFFFFFFFF]
        assert store([(1, "e", 7), (1, "f", [1, 2])]) == [1, 4]
        got = tset.run(["{a}", "{d}", "{e}", "{f}", "{b}"], [0, 1, 1, 1, 0])
        assert got[0] == (N.OK_VALUE, 0) and got[1] == (N.OK_VALUE, 3) and got[2] == (N.OK_VALUE, 1)
        assert got[3] == (N.OK_VALUE, 4) and got[4][0] == N.E_INTERP
    finally:
        tset.close()


def test_update_keeps_values_by_store_ids():
    # the mirror's update goes through ie_table_set_store: typed whole-string results after rewrites,
    # deletes and re-adds come back as the stored objects
    states = [{"n": 1, "s": "x"} for _ in range(50)]
    tset = IE.InsertsTableSet(states, clock=CLOCK, mutable=True)
    try:
        for rnd in range(4):
            changes = []
            for t in range(50):
                if (t + rnd) % 3 == 0:
                    changes.append((t, "n", IE.DELETE))
                    states[t].pop("n", None)
                else:
                    changes.append((t, "n", [rnd, t]))
                    states[t]["n"] = [rnd, t]
                changes.append((t, "k%d" % rnd, {"r": rnd}))
                states[t]["k%d" % rnd] = {"r": rnd}
            assert tset.update(changes)
            res = tset.results(["{n}" for _ in range(50)] + ["{k%d}" % rnd for _ in range(50)], list(range(50)) * 2)
            for t in range(50):
                want = states[t].get("n")
                if want is None:
                    assert isinstance(res[t], IE.InterpolationException)
                else:
                    assert res[t] == want
                assert res[50 + t] == {"r": rnd}
    finally:
        tset.close()


def test_large_rewrite_batches_match_the_oracle():
    # >= 4096 stores that only rewrite present keys take the parallel placement (per-thread arena
    # regions): shorter texts in place, longer ones appended, a key stored twice in one call (the
    # second wins), typed values; every string matches the oracle on the mutated states after each
    # round, and the value ids stay those of the keys
    rng = random.Random(9)
    states = [{"h": "hist %d" % t, "o": "out", "n": t, "tmpl": "<{h}|{o}>"} for t in range(2000)]
    tset = IE.InsertsTableSet(states, clock=CLOCK, mutable=True)
    try:
        # the first round reverts the pre-resolved templates (serial path); the next ones are rewrites only
        for rnd in range(4):
            changes = []
            for t, d in enumerate(states):
                d["h"] = d["h"] + " more %d" % rnd * rng.randrange(0, 6)
                d["o"] = "o%d" % rng.randrange(0, 10 ** rng.randrange(1, 6))
                d["n"] = d["n"] + rnd
                changes += [(t, "h", d["h"]), (t, "o", "ignored"), (t, "o", d["o"]), (t, "n", d["n"])]
            before = [tset.run(["{n}"], [t])[0][1] for t in (0, 777)]
            assert tset.update(changes)
            strings = ["{h}", "x{o}y", "{tmpl}", "{n}", "n={n}"] * len(states)
            ids = [t for t in range(len(states)) for _ in range(5)]
            bad = _check(tset, states, strings, ids)
            assert not bad, (rnd, len(bad), bad[:3])
            assert [tset.run(["{n}"], [t])[0][1] for t in (0, 777)] == before  # ids kept by rewrites
            size, live, _ = tset.arena_stats()
            assert size <= 2 * live + (64 << 10) + 64 or rnd == 0, (rnd, size, live)
    finally:
        tset.close()


def test_value_reads_from_two_threads():
    """ie_table_value's value-id -> slot map is rebuilt lazily after an update, on the read path;
    ctypes releases the GIL, so two threads reading one table's values at once both reach that
    rebuild (the header: a table may be read by several threads). Every read must still return
    the stored value."""
    import threading
    states = [{"k%d" % j: "v%d-%d" % (t, j) for j in range(40)} for t in range(200)]
    tset = IE.InsertsTableSet(states, clock=CLOCK, mutable=True)
    try:
        errors = []
        for rnd in range(5):
            changes = [(t, "k%d" % ((t + rnd) % 40), "w%d-%d" % (rnd, t)) for t in range(200)]
            assert tset.update(changes)
            for t, k, v in changes:
                states[t][k] = v
            vids = [(tset.keys.index(k, tset.starts[t], tset.starts[t + 1]), states[t][k])
                    for t in range(200) for k in ("k%d" % ((t + rnd) % 40), "k%d" % ((t + rnd + 1) % 40))]

            def read(part):
                try:
                    for vid, want in part:
                        got = tset.value(vid)
                        if got != want:
                            errors.append((vid, got, want))
                except Exception as e:  # noqa: BLE001 (reported below)
                    errors.append(repr(e))
            ths = [threading.Thread(target=read, args=(vids[i::2],)) for i in range(2)]
            for th in ths:
                th.start()
            for th in ths:
                th.join()
        assert not errors, errors[:3]
    finally:
        tset.close()


def test_deleted_keys_give_their_value_ids_back():
    """delete / delete_except through ie_delete_keys (the store path): each deleted key's value id
    is reported, goes back to the set's free list (the next new key takes it) and the mirror drops
    the value it held under it."""
    from interpolation_engine_amd import maps as M
    states = [{"keep": "a", "drop_1": "b", "drop_2": [1, 2]} for _ in range(30)]
    tset = IE.InsertsTableSet(states, clock=CLOCK, mutable=True)
    try:
        got = M.delete_states(states, {"cmd": "delete", "wildcards": ["drop_*"]}, tables=tset)
        assert all(sorted(g) == ["drop_1", "drop_2"] for g in got)
        assert all(set(s) == {"keep"} for s in states)
        freed = [i for i, v in enumerate(tset.values) if v is None]
        assert len(freed) == 60  # (the typed list values are no longer held)
        assert tset.update([(0, "new", [3])])
        r = tset.run(["{new}"], [0])[0]
        assert r[0] == N.OK_VALUE and r[1] in freed and tset.value(r[1]) == [3]
    finally:
        tset.close()
