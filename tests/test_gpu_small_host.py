"""The small-batch host path (ie_host.cpp run_host_small: inputs in one pinned block, every output
array back with one copy, one synchronisation) against the per-array path (IE_SMALL_HOST=0) and the
C oracle on the same batches: identical statuses, bytes and value ids, packed and views, with table
ids, and with an output larger than the small path's first-guess capacity (it hands the batch to the
per-array path)."""
import random

import pytest

import __graft_entry__ as G
from oracle import oracle as O

pytestmark = pytest.mark.gpu

G.build()
PKG = G.load_package()
N = PKG._native
CLOCK = (7, 8, 9)


def _exec(monkeypatch, small, views):
    monkeypatch.setenv("IE_SMALL_HOST", "1" if small else "0")
    x = N.Exec(0)
    x.set_option(N.OPT_VIEWS, views)
    return x


def _batch(rng, n):
    keys = ["k%d" % j for j in range(40)]
    out = []
    for _ in range(n):
        parts = []
        for _ in range(rng.randrange(0, 4)):
            r = rng.random()
            if r < 0.5:
                parts.append("{%s}" % rng.choice(keys))
            elif r < 0.7:
                parts.append("{n-{%s}}" % rng.choice(keys[:8]))
            elif r < 0.8:
                parts.append("{missing%d}" % rng.randrange(5))
            elif r < 0.9:
                parts.append("\\{lit\\}")
            else:
                parts.append("{big}")
            parts.append("".join(rng.choice("abc xyz") for _ in range(rng.randrange(0, 12))))
        out.append("".join(parts))
    return out


TABLE = dict({"k%d" % j: "v%d" % j for j in range(40)}, **{"n-v%d" % j: "nested%d" % j for j in range(8)},
             big="B" * 3000, num=17)


@pytest.mark.parametrize("views", [0, 1])
@pytest.mark.parametrize("n", [1, 7, 300, 1024])
def test_small_path_matches_per_array_path(monkeypatch, views, n):
    rng = random.Random(1000 * n + views)
    strings = _batch(rng, n)
    t = PKG.InsertsTable(TABLE, clock=CLOCK)
    small = t.run(strings, exec_=_exec(monkeypatch, True, views))
    generic = t.run(strings, exec_=_exec(monkeypatch, False, views))
    assert small == generic
    ref = O.Oracle(TABLE, "py", clock=CLOCK)
    for s, (st, payload) in zip(strings, small):
        rst, rout, _ = ref.interpolate(s)
        assert N.STATUS_NAMES[st] == rst, s
        if rst == "OK_STR":
            assert payload == rout, s


@pytest.mark.parametrize("views", [0, 1])
def test_small_path_output_past_first_capacity(monkeypatch, views):
    # 12 x 3000 bytes of output from a 60-byte input: more than 2 x input + 4096
    strings = ["{big}" * 12, "x{k1}y"]
    t = PKG.InsertsTable(TABLE, clock=CLOCK)
    got = t.run(strings, exec_=_exec(monkeypatch, True, views))
    assert got == [(N.OK_STR, "B" * 36000), (N.OK_STR, "xv1y")]


def test_small_path_table_ids(monkeypatch):
    dicts = [{"a": "A%d" % i, "b": "{a}-%d" % i} for i in range(5)]
    ts = PKG.InsertsTableSet(dicts, clock=CLOCK)
    rng = random.Random(5)
    strings = [rng.choice(["{a}", "<{b}>", "{c}", "t{a}{b}"]) for _ in range(200)]
    ids = [rng.randrange(5) for _ in strings]
    small = ts.run(strings, ids, exec_=_exec(monkeypatch, True, 0))
    generic = ts.run(strings, ids, exec_=_exec(monkeypatch, False, 0))
    assert small == generic
    for s, i, (st, payload) in zip(strings, ids, small):
        rst, rout, _ = O.Oracle(dicts[i], "py", clock=CLOCK).interpolate(s)
        assert N.STATUS_NAMES[st] == rst, (s, i)
        if rst == "OK_STR":
            assert payload == rout, (s, i)


@pytest.mark.parametrize("zc", [1, 2])
def test_small_path_without_copies(monkeypatch, zc):
    """IE_OPT_SMALL_ZC (run_host_small_zc): one-tile views calls read and write a mapped host block
    and k_resolve leaves the call's counters zeroed for the next one; calls in a row, between them
    calls on the other paths (a 300-string batch, an output past the first-guess capacity, which
    leave the zero-copy counters to the host), each equal to the copying path and the oracle."""
    rng = random.Random(77 + zc)
    t = PKG.InsertsTable(TABLE, clock=CLOCK)
    x = _exec(monkeypatch, True, 1)
    x.set_option(N.OPT_SMALL_ZC, zc)
    ref_x = _exec(monkeypatch, True, 1)
    ref = O.Oracle(TABLE, "py", clock=CLOCK)
    for k, n in enumerate([1, 1, 7, 256, 300, 1, ("{big}" * 12,), 3, 200, 1]):
        strings = list(n) if isinstance(n, tuple) else _batch(rng, n)
        got = t.run(strings, exec_=x)
        assert got == t.run(strings, exec_=ref_x), k
        for s, (st, payload) in zip(strings, got):
            rst, rout, _ = ref.interpolate(s)
            assert N.STATUS_NAMES[st] == rst, (k, s)
            if rst == "OK_STR":
                assert payload == rout, (k, s)
    with pytest.raises(RuntimeError):
        x.set_option(N.OPT_SMALL_ZC, 3)


def test_small_wildcard_batch_without_copies(monkeypatch):
    """ie_wildcard_match_batch's small batch in the mapped block (IE_OPT_SMALL_ZC): the same matches
    and captures as with the block copies."""
    from interpolation_engine_amd.wildcard import Wildcards
    pats = ["go *", "take * from *", "*"]
    texts = ["go north", "take lamp from table", "look", "take x from y", "go  "] * 9
    w = Wildcards(pats)
    try:
        got = []
        for zc in (0, 1):
            x = _exec(monkeypatch, True, 1)
            x.set_option(N.OPT_SMALL_ZC, zc)
            match, ncap, caps = w.match_raw(texts, None, exec_=x)
            # (capture slots past a string's count are not written: compared up to the count)
            got.append((match.tolist(), ncap.tolist(), [caps[i, :ncap[i]].tolist() for i in range(len(texts))]))
    finally:
        w.close()
    assert got[0] == got[1]
    assert got[0][0][:3] == [0, 1, 2]
