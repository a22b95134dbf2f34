"""Parity of the HIP path (through the C ABI of libie_amd.so) with the reference.

Checkers: the reference's own golden vectors (tests/golden/, generated from the reference Python
module) and the C oracle (oracle/ie_oracle.c, itself pinned by those vectors in
test_oracle_golden.py). Bar: byte-identical strings, identical status class, identical typed
value (same insert) — bit-exact, this is byte/index work.
"""
import ctypes
import os
import random

import numpy as np
import pytest

import __graft_entry__ as G
from oracle import oracle as O
from tests.conftest import load_golden

pytestmark = pytest.mark.gpu

G.build()
PKG = G.load_package()
N = PKG._native
CLOCK = (12, 34, 56)
VID_SPECIAL = {"@HH:MM": N.VID_HHMM, "@HH:MM:SS": N.VID_HHMMSS}


def run_product(table_dict, strings, dialect="py", has_dir=False):
    t = PKG.InsertsTable(table_dict, dialect=dialect, clock=CLOCK, has_inserts_dir=has_dir)
    return t.run(strings), t


@pytest.fixture(params=["0", "1", "1w", "0v", "1v", "0rv", "1rv", "0dv", "1dv"],
                ids=["chain-fail-exact", "chain-fail-commit", "chain-fail-commit-512", "chain-fail-exact-views",
                     "chain-fail-commit-views", "chain-fail-exact-views-reserve", "chain-fail-commit-views-reserve",
                     "chain-fail-exact-views-defer", "chain-fail-commit-views-defer"])
def fail_commit(request, monkeypatch):
    """Both k_resolve variants: chain failures sent to the exact evaluator, or committed in the
    chain evaluator (the library picks one adaptively; IE_FAIL_COMMIT / IE_OPT_FAIL_COMMIT force it);
    also with 512-string tiles (ie_resolve512.hip, IE_OPT_TILE) and with the views output layout
    (no look-back; IE_OPT_VIEWS, packed on the host by the batch API; _device_run uses
    ie_interpolate_device_views). Execs read the environment when they are created; the mirror's
    cached exec is set directly. Yields the fail-commit digit; VIEWS[0] tells _device_run."""
    fc, tile = request.param[0], 512 if request.param.endswith("w") else 0
    views = 1 if request.param.endswith("v") else 0
    # reserved output ranges (IE_OPT_RESERVE: tiles write at 2x their input offsets, no claim atomic;
    # ie_interpolate_device_views only)
    reserve = 32 if "r" in request.param else 0
    defer = 1 if "d" in request.param else 0  # heavy strings to a second pass (IE_OPT_DEFER)
    monkeypatch.setenv("IE_RESERVE", str(reserve))
    monkeypatch.setenv("IE_DEFER", str(defer))
    monkeypatch.setenv("IE_FAIL_COMMIT", fc)
    monkeypatch.setenv("IE_TILE", str(tile))
    monkeypatch.setenv("IE_VIEWS", str(views))
    x = PKG.interpolation_engine.get_exec(0)
    x.set_option(N.OPT_FAIL_COMMIT, int(fc))
    x.set_option(N.OPT_TILE, tile)
    x.set_option(N.OPT_VIEWS, views)
    x.set_option(N.OPT_RESERVE, reserve)
    x.set_option(N.OPT_DEFER, defer)
    VIEWS[0] = bool(views)
    yield fc
    VIEWS[0] = False
    x.set_option(N.OPT_RESERVE, 0)
    x.set_option(N.OPT_DEFER, -1)
    x.set_option(N.OPT_FAIL_COMMIT, -1)
    x.set_option(N.OPT_TILE, 0)
    x.set_option(N.OPT_VIEWS, 0)


VIEWS = [False]  # set by the fail_commit fixture: device runs use the views layout


def compare_with_oracle(table_dict, strings, dialect="py", has_dir=False):
    got, t = run_product(table_dict, strings, dialect, has_dir)
    ref = O.Oracle(table_dict, dialect, clock=CLOCK, has_dir=has_dir)
    bad = []
    for s, (st, payload) in zip(strings, got):
        rst, rout, rvid = ref.interpolate(s)
        name = N.STATUS_NAMES[st]
        ok = name == rst
        if ok and rst == "OK_STR":
            ok = payload == rout
        if ok and rst == "OK_VALUE":
            ok = payload == rvid
        if not ok:
            bad.append((s, name, payload, rst, rout, rvid))
    return bad


# ------------------------------------------------------------------------------------------
# golden vectors from the reference itself
# ------------------------------------------------------------------------------------------
def test_reference_golden_vectors(golden_tables, golden_interp, fail_commit):
    by_table = {}
    for row in golden_interp:
        by_table.setdefault(row["t"], []).append(row)
    bad = []
    for ti, rows in by_table.items():
        got, t = run_product(golden_tables[ti], [r["s"] for r in rows])
        for row, (st, payload) in zip(rows, got):
            name = N.STATUS_NAMES[st]
            ok = name == row["st"]
            if ok and name == "OK_STR":
                ok = payload == row["out"]
            if ok and name == "OK_VALUE":
                want = {VID_SPECIAL.get(k, t.keys.index(k) if k in t.keys else -1) for k in row["vkeys"]}
                ok = payload in want
            if not ok:
                bad.append((ti, row, name, payload))
    assert not bad, "%d mismatches; first %r" % (len(bad), bad[:4])


def test_rust_dialect_matches_restated_oracle(golden_tables, golden_interp):
    """Rust dialect (parity unpinned: the crate cannot be built here) vs the oracle's restatement."""
    by_table = {}
    for row in golden_interp:
        by_table.setdefault(row["t"], []).append(row["s"])
    for ti, strings in by_table.items():
        bad = compare_with_oracle(golden_tables[ti], strings, "rs")
        assert not bad, bad[:4]


def test_inserts_dir_statuses(golden_tables, golden_interp):
    strings = [r["s"] for r in golden_interp if r["t"] == 0]
    bad = compare_with_oracle(golden_tables[0], strings, "py", has_dir=True)
    assert not bad, bad[:4]


# ------------------------------------------------------------------------------------------
# randomized differential tests against the oracle
# ------------------------------------------------------------------------------------------
def _rand_table(rng, n, brace_values):
    t = {}
    for j in range(n):
        k = "k%d" % j
        r = rng.random()
        if r < 0.6:
            v = "".join(rng.choice("abcxyz é€😀-.") for _ in range(rng.randint(0, 12)))
            if brace_values and rng.random() < 0.3:
                v += "{k%d}" % rng.randrange(n)
            if rng.random() < 0.05:
                v += "\\"
            if rng.random() < 0.05:
                v = "\\}" + v
        elif r < 0.8:
            v = rng.randint(-10**6, 10**6)
        elif r < 0.9:
            v = ["a", rng.randint(0, 9)]
        else:
            v = rng.choice([1.25, True, None, {"z": 1}])
        t[k] = v
    t["q-"] = "Q"
    return t


def _rand_string(rng, n_keys, long=False):
    parts = []
    for _ in range(rng.randint(0, 40 if long else 8)):
        r = rng.random()
        if r < 0.35:
            parts.append("".join(rng.choice("abc .,é😀\n") for _ in range(rng.randint(1, 30 if long else 6))))
        elif r < 0.7:
            parts.append("{k%d}" % rng.randrange(n_keys + 3))
        elif r < 0.8:
            parts.append("{q-{k%d}}" % rng.randrange(n_keys))
        elif r < 0.85:
            parts.append("{" * 7 + "k1" + "}" * 7)
        elif r < 0.9:
            parts.append(rng.choice(["\\{", "\\}", "\\{lit\\}", "\\", ".\\}", "〠", "}", "{"]))
        else:
            parts.append("{k%d-" % rng.randrange(n_keys) + "x" * rng.randint(0, 60) + "}")
    s = "".join(parts)
    if rng.random() < 0.1:
        s = "{" + s + "}"
    return s


@pytest.mark.parametrize("dialect", ["py", "rs"])
def test_chain_failures_follow_the_reference_order(dialect, fail_commit):
    """Misses and unspliceable hits inside chain-shaped strings: the reference reports the failing
    pair with the largest opening offset (rightmost chain, innermost level) and never evaluates
    the pairs enclosing it."""
    table = {"a": "A", "i": 2, "q-2": "Q2", "f": 1.5, "n": None, "d": {"z": 1}, "L": ["x", 1], "b": True,
             "q-A": "QA", "q-1.5": "QF", "i2": "f"}
    pieces = ["{a}", "{zz}", "{f}", "{n}", "{d}", "{L}", "{b}", "{q-{i}}", "{q-{zz}}", "{q-{f}}", "{zz-{a}}",
              "{q-{a}}", "{{i2}}", "{q-{q-{i}}}", "{}", "x", "é"]
    rng = random.Random(11)
    strings = ["x{zz}{f}", "x{f}{zz}", "x{q-{zz}}{a}", "x{a}{q-{f}}", "x{zz-{f}}", "x{q-{f}}y{zz}",
               "x{zz}y{q-{n}}", "{q-{zz}}", "x{}{a}"]
    for _ in range(4000):
        strings.append("".join(rng.choice(pieces) for _ in range(rng.randint(1, 4))))
    bad = compare_with_oracle(table, strings, dialect)
    assert not bad, bad[:4]


@pytest.mark.parametrize("dialect", ["py", "rs"])
def test_escapes_next_to_chains(dialect, fail_commit):
    """Escaped braces inside chain-shaped strings (the chain evaluator treats a brace after '\\' as
    text) and the restore hazards that must leave it: '\\}' after '.', after a real '}' (a value
    may end in '.') and after another '\\}'; backslash runs; escapes inside keys."""
    table = {"k1": "V1", "k2": "dot.", "q-3": "Q3", "i": 3, "a\\}b": "AB", "a\\{b": "AB2", "x.": "XD",
             "\\{": "BR", "q-V1": "QV"}
    pieces = ["{k1}", "{k2}", "{q-{i}}", "\\{", "\\}", ".", "\\", "x", "{a\\}b}", "{a\\{b}", "}", "{",
              "{q-{k1}}", "é", "{\\{}"]
    rng = random.Random(7)
    strings = ["a.\\}b{k1}", "{k1}\\}x", "{k2}\\}x", "\\}\\}{k1}", "\\{k1\\}{k2}", "x\\{{k1}\\}",
               "{a\\}b}", "\\\\{k1}", "\\\\}{k1}", ".\\{{k1}", "{k1}.\\}", "\\}{k1}", "p{k1}\\",
               "{a\\{b}{q-{i}}\\{", "z{\\{}z"]
    for _ in range(4000):
        strings.append("".join(rng.choice(pieces) for _ in range(rng.randint(1, 9))))
    bad = compare_with_oracle(table, strings, dialect)
    assert not bad, bad[:4]


@pytest.mark.parametrize("dialect", ["py", "rs"])
def test_preresolved_values_keep_raw_lookups(dialect):
    """Brace-bearing values are pre-resolved at table build (splice text = their resolution) while
    whole-string lookups by value (py:512 / interp.rs:48) still see the raw value: keys equal to
    both the raw and the resolved text tell the two apart."""
    table = {"a": "{b}", "b": "x{c}y", "c": "C", "x{c}y": "raw-hit", "xCy": "resolved-hit",
             "d": "<{b}|{c}>", "e": "{a}{a}", "loop": "{loop}", "m": "{nope}", "n": 7, "w": "{n}",
             "esc": "\\{b\\}", "half": "}{", "deep": "{e}{d}{e}"}
    strings = ["{a}", "{{a}}", "{{b}}", "{{{b}}}", "z{b}z", "{x{c}y}", "<{d}>", "{e}", "e={e}!", "{loop}",
               "x{loop}", "x{m}", "{m}", "{{m}}", "w{w}", "{w}", "{{w}}", "{esc}", "-{esc}-", "{half}",
               "-{half}-", "{deep}", "a{deep}b{a}", "\\{a\\}{a}", "{q-{c}}", "{x{a}y}"]
    bad = compare_with_oracle(table, strings, dialect)
    assert not bad, bad[:4]


@pytest.mark.parametrize("seed,brace_values,dialect", [(1, False, "py"), (2, True, "py"), (3, False, "rs"),
                                                       (4, True, "rs")])
def test_random_vs_oracle(seed, brace_values, dialect, fail_commit):
    rng = random.Random(seed)
    table = _rand_table(rng, 60, brace_values)
    strings = [_rand_string(rng, 60) for _ in range(3000)]
    bad = compare_with_oracle(table, strings, dialect)
    assert not bad, bad[:4]


def test_long_strings_and_oversized_tiles():
    """Tiles above the LDS stage (long strings) take the global-memory path."""
    rng = random.Random(7)
    table = _rand_table(rng, 40, False)
    strings = [_rand_string(rng, 40, long=True) for _ in range(700)]
    strings += ["x" * 5000 + "{k1}" + "y" * 3000, "{k2}" * 2000, "a" * 70000]
    bad = compare_with_oracle(table, strings)
    assert not bad, [b[:2] for b in bad[:4]]


def _chain_table():
    t = {}
    for d in range(10):
        t["x%d" % d] = str(d)
        t["a-%d" % d] = str(d)
        t["a-%dz" % d] = str((d + 1) % 10)
        t["q%d" % d] = "v%d é" % d
    return t


def _chain(rng, depth):
    s = "x%d" % (rng.randrange(10) if rng.random() < 0.97 else 10)  # x10: an innermost miss
    for _ in range(depth - 1):
        s = "{" + s + "}"
        pre = "a-" if rng.random() < 0.97 else "b-"  # b-: a miss at an outer level
        s = pre + s + rng.choice(["", "", "z"])
    return "{" + s + "}"


@pytest.mark.parametrize("n_keys", [6000, 30000, 130000])
def test_table_sizes_vs_oracle(n_keys):
    """Pilot placement regimes: ~4 keys per group in LDS (6k keys), up to 20 per group in LDS
    (30k), and a table too large for the LDS copy whose pilots are read from L2 (130k)."""
    rng = random.Random(n_keys)
    table = {"k%d" % j: ("v%d" % j if j % 3 else j) for j in range(n_keys)}
    table.update({"q-%d" % j: "Q%d é" % j for j in range(n_keys // 4)})
    strings = []
    for _ in range(3000):
        parts = ["x "]
        for _ in range(rng.randint(1, 3)):
            r = rng.random()
            if r < 0.5:
                parts.append("{k%d}" % rng.randrange(n_keys + 50))
            else:
                parts.append("{q-{k%d}}" % rng.randrange(n_keys // 4))
            parts.append(" . ")
        strings.append("".join(parts))
    bad = compare_with_oracle(table, strings)
    assert not bad, bad[:4]


@pytest.mark.parametrize("seed", [11, 12])
def test_deep_chains_vs_oracle(seed):
    """Chains of depth 1-5 ({a-{a-{x3}z}}...): the chain evaluator's middle levels, misses at
    every level, up to three chains per string, and depth 5 (exact evaluator)."""
    rng = random.Random(seed)
    strings = []
    for _ in range(4000):
        parts = [rng.choice(["", "t ", "é-", "text. "])]
        for _ in range(rng.randint(1, 3)):
            parts.append(_chain(rng, rng.choice([1, 2, 3, 4, 4, 5])))
            parts.append(rng.choice(["", " ", " and ", "😀"]))
        strings.append("".join(parts))
    bad = compare_with_oracle(_chain_table(), strings)
    assert not bad, bad[:4]


@pytest.mark.parametrize("n", [0, 1, 255, 256, 257, 511, 1000])
def test_batch_sizes(n):
    rng = random.Random(n)
    table = _rand_table(rng, 30, False)
    strings = [_rand_string(rng, 30) for _ in range(n)]
    bad = compare_with_oracle(table, strings)
    assert not bad, bad[:4]


def test_runaway_inserts_diverge_like_the_oracle():
    table = {"a": "{a}", "g": "{g}{g}", "s": "x{s}", "ok": "fine"}
    strings = ["x{a}", "x{g}", "{s}", "y{s}", "x{ok}", "{a}"]
    bad = compare_with_oracle(table, strings)
    assert not bad, bad


def test_large_growth_retries_scratch():
    """A value that expands far beyond the default literal scratch: the host API retries."""
    table = {"big": "{w}" * 50, "w": "word-" * 40 + "{x}", "x": "X" * 100}
    strings = ["a{big}b", "{big}", "c{w}d"]
    bad = compare_with_oracle(table, strings)
    assert not bad, [b[:2] for b in bad]


# ------------------------------------------------------------------------------------------
# the synthetic benchmark configs
# ------------------------------------------------------------------------------------------
def _synth(config):
    h = ctypes.c_void_p()
    N.check(N.lib().ie_synth_create(config, 0, ctypes.byref(h)), "ie_synth_create")
    kvp = ctypes.POINTER(N.KV)()
    nkv = N.lib().ie_synth_kv(h, ctypes.byref(kvp))
    return h, kvp, nkv


def _table_from_kv(kvp, nkv, clock=CLOCK):
    t = ctypes.c_void_p()
    clk = N.Clock(*clock)
    N.check(N.lib().ie_table_build(ctypes.cast(kvp, ctypes.c_void_p), nkv, 0, ctypes.byref(clk), 0, 0,
                                   ctypes.byref(t)), "ie_table_build")
    return t


def _host_strings(h, first, n):
    offs = np.zeros(n + 1, np.uint64)
    total = ctypes.c_uint64()
    N.check(N.lib().ie_synth_strings_host(h, first, n, None, 0, offs.ctypes.data, ctypes.byref(total)), "len")
    buf = np.zeros(int(total.value) + 1, np.uint8)
    N.check(N.lib().ie_synth_strings_host(h, first, n, buf.ctypes.data, buf.size, offs.ctypes.data,
                                          ctypes.byref(total)), "fill")
    return buf, offs


@pytest.mark.parametrize("config", [2, 3, 4])
def test_device_synth_equals_host_synth(config):
    h, kvp, nkv = _synth(config)
    x = N.Exec(0)
    n = 100_000
    buf, offs = _host_strings(h, 12345, n)
    d_off, d_bytes, total = _device_strings(x, h, 12345, n)
    assert np.array_equal(d_off.to_numpy(np.uint64, n + 1), offs)
    assert np.array_equal(d_bytes.to_numpy(np.uint8, total), buf[:total])


def _device_strings(x, h, first, n):
    d_off = N.DeviceBuffer(x, (n + 1) * 8)
    total = ctypes.c_uint64()
    N.check(N.lib().ie_synth_strings_device(x.h, h, first, n, None, 0, d_off.ptr, ctypes.byref(total)), "d")
    d_bytes = N.DeviceBuffer(x, int(total.value) + 16)
    N.check(N.lib().ie_synth_strings_device(x.h, h, first, n, d_bytes.ptr, d_bytes.nbytes, d_off.ptr,
                                            ctypes.byref(total)), "d")
    return d_off, d_bytes, int(total.value)


class DevResult:
    def __init__(self, x, n, cap):
        self.n = n
        self.bytes = N.DeviceBuffer(x, cap)
        self.off = N.DeviceBuffer(x, (n + 1) * 8)
        self.status = N.DeviceBuffer(x, n + 1)
        self.vid = N.DeviceBuffer(x, 4 * n + 4)
        self.total_d = N.DeviceBuffer(x, 8)
        self.out = N.DevOut(self.bytes.ptr, cap, self.off.ptr, self.status.ptr, self.vid.ptr, self.total_d.ptr)

    def total(self):
        return int(self.total_d.to_numpy(np.uint64, 1)[0])


def assert_views_disjoint(starts, lens, total):
    """A views output: every result inside [0, total) and no two overlapping (reserved ranges leave
    gaps between tiles, so `total` here is the extent the caller read back, at least the sum of the
    lengths)."""
    starts, lens = np.asarray(starts, np.int64), np.asarray(lens, np.int64)
    nz = lens > 0
    s, l = starts[nz], lens[nz]
    assert np.all(s + l <= total) and int(l.sum()) <= total
    o = np.argsort(s, kind="stable")
    assert np.all(s[o][1:] >= (s[o] + l[o])[:-1])


def _device_run(x, table, d_bytes, d_off, n, cap=None):
    """A packed result; with the views fixture the device writes views, packed here on the host in
    input order (the check then runs on the same packed form)."""
    r = DevResult(x, n, cap if cap is not None else int(d_bytes.nbytes * 3 + 4096))
    if not VIEWS[0]:
        N.check(N.lib().ie_interpolate_device(x.h, table, d_bytes.ptr, d_off.ptr, n, ctypes.byref(r.out)),
                "ie_interpolate_device")
        x.sync()
        return r
    lens = N.DeviceBuffer(x, 4 * n + 4)
    v = N.DevViews(r.bytes.ptr, r.out.bytes_cap, r.off.ptr, lens.ptr, r.status.ptr, r.vid.ptr, r.total_d.ptr)
    N.check(N.lib().ie_interpolate_device_views(x.h, table, None, d_bytes.ptr, d_off.ptr, None, n, ctypes.byref(v)),
            "ie_interpolate_device_views")
    x.sync()
    tot = r.total()
    starts = r.off.to_numpy(np.uint64, n)
    ln = lens.to_numpy(np.uint32, n).astype(np.uint64)
    assert int(ln.sum()) == tot  # *total = sum of lengths (reserved ranges: gaps between tiles)
    ext = int((starts + ln).max()) if n else 0
    blob = r.bytes.to_numpy(np.uint8, max(ext, tot))
    assert_views_disjoint(starts, ln, blob.size)
    packed = np.concatenate([blob[int(starts[i]):int(starts[i] + ln[i])] for i in range(n)]) if n else blob
    offs = np.zeros(n + 1, np.uint64)
    offs[1:] = np.cumsum(ln)
    r.bytes = N.DeviceBuffer.from_numpy(x, np.concatenate([packed, np.zeros(16, np.uint8)]))
    r.off = N.DeviceBuffer.from_numpy(x, offs)
    r.total_d = N.DeviceBuffer.from_numpy(x, offs[-1:].copy())  # the packed form's total
    return r


@pytest.mark.parametrize("config", [2, 3, 4])
def test_synthetic_config_vs_oracle(config, fail_commit):
    h, kvp, nkv = _synth(config)
    table = _table_from_kv(kvp, nkv)
    x = N.Exec(0)
    n = 200_000
    buf, offs = _host_strings(h, 0, n)
    d_bytes = N.DeviceBuffer.from_numpy(x, buf)
    d_off = N.DeviceBuffer.from_numpy(x, offs)
    r = _device_run(x, table, d_bytes, d_off, n)
    ref = O.Oracle.from_kv(ctypes.cast(kvp, ctypes.c_void_p), nkv, "py", clock=CLOCK)
    rst = np.zeros(n, np.uint8)
    rlen = np.zeros(n, np.uint64)
    rhash = np.zeros(n, np.uint64)
    ref.run_batch(buf, offs, n, 8, rst, rlen, rhash, None)
    st = r.status.to_numpy(np.uint8, n)
    oo = r.off.to_numpy(np.uint64, n + 1)
    total = r.total()
    ob = r.bytes.to_numpy(np.uint8, total).tobytes()
    assert np.array_equal(st, rst)
    assert np.array_equal(np.diff(oo.astype(np.int64)), rlen.astype(np.int64))
    # the oracle hashes OK_STR outputs only (0 for status rows)
    hashes = np.array([O.fnv1a(ob[int(oo[i]):int(oo[i + 1])]) if st[i] == 0 else 0 for i in range(n)],
                      dtype=np.uint64)
    assert np.array_equal(hashes, rhash)
    N.lib().ie_table_free(table)


def test_full_size_config3_properties():
    """Config 3 at its BASELINE size (10M strings): size-independent properties + a sampled
    oracle check. Properties: every status OK_STR, offsets monotone with the right total, no
    brace left in any output, idempotence (re-resolving the outputs is the identity)."""
    h, kvp, nkv = _synth(3)
    table = _table_from_kv(kvp, nkv)
    x = N.Exec(0)
    n = 10_000_000
    d_off, d_bytes, in_total = _device_strings(x, h, 0, n)
    r = _device_run(x, table, d_bytes, d_off, n)
    tot = r.total()
    st = r.status.to_numpy(np.uint8, n)
    assert int(np.count_nonzero(st)) == 0
    oo = r.off.to_numpy(np.uint64, n + 1)
    lens = np.diff(oo.astype(np.int64))
    assert lens.min() >= 0 and int(oo[-1]) == tot
    ob = r.bytes.to_numpy(np.uint8, tot)
    assert int(np.count_nonzero(ob == ord("{"))) == 0 and int(np.count_nonzero(ob == ord("}"))) == 0
    # idempotence: the outputs are brace-free, so resolving them again changes nothing
    r2 = _device_run(x, table, r.bytes, r.off, n)
    assert r2.total() == tot
    assert np.array_equal(r2.off.to_numpy(np.uint64, n + 1), oo)
    assert np.array_equal(r2.bytes.to_numpy(np.uint8, tot), ob)
    # sampled oracle check across the whole index range
    rng = np.random.default_rng(0)
    ref = O.Oracle.from_kv(ctypes.cast(kvp, ctypes.c_void_p), nkv, "py", clock=CLOCK)
    for i in np.sort(rng.choice(n, 500, replace=False)):
        b, o = _host_strings(h, int(i), 1)
        rs, rout, _ = ref.interpolate(b[:int(o[1])].tobytes())
        assert rs == "OK_STR"
        assert ob[int(oo[i]):int(oo[i + 1])].tobytes().decode("utf-8") == rout
    N.lib().ie_table_free(table)


def _unescape_cmd(x, table, r, n, cap):
    """The `unescape` command (py:1660-1667) over a resolved batch r: recursive_unescape, then
    recursive_interpolate; strings that failed in r keep their status."""
    tmp = DevResult(x, n, cap)
    out = DevResult(x, n, cap)
    N.check(N.lib().ie_unescape_cmd_device(x.h, table, None, r.bytes.ptr, r.off.ptr, n, r.status.ptr,
                                           ctypes.byref(tmp.out), ctypes.byref(out.out)), "ie_unescape_cmd_device")
    x.sync()
    return tmp, out


def test_config4_step_vs_oracle(fail_commit):
    """Config 4's whole step on 200k strings, string for string against the oracle running
    interpolate, then the unescape command (unescape, interpolate again: py:1660-1667)."""
    h, kvp, nkv = _synth(4)
    table = _table_from_kv(kvp, nkv)
    x = N.Exec(0)
    n = 200_000
    buf, offs = _host_strings(h, 5_000_000, n)
    d_bytes = N.DeviceBuffer.from_numpy(x, buf)
    d_off = N.DeviceBuffer.from_numpy(x, offs)
    r = _device_run(x, table, d_bytes, d_off, n)
    _, u = _unescape_cmd(x, table, r, n, 2 * r.total() + 4096)
    ref = O.Oracle.from_kv(ctypes.cast(kvp, ctypes.c_void_p), nkv, "py", clock=CLOCK)
    rst = np.zeros(n, np.uint8)
    rlen = np.zeros(n, np.uint64)
    rhash = np.zeros(n, np.uint64)
    ref.run_batch(buf, offs, n, 8, rst, rlen, rhash, None, unescape_cmd=True)
    st = u.status.to_numpy(np.uint8, n)
    oo = u.off.to_numpy(np.uint64, n + 1)
    ob = u.bytes.to_numpy(np.uint8, u.total()).tobytes()
    assert np.array_equal(st, rst)
    assert np.array_equal(np.diff(oo.astype(np.int64)), rlen.astype(np.int64))
    hashes = np.array([O.fnv1a(ob[int(oo[i]):int(oo[i + 1])]) if st[i] == 0 else 0 for i in range(n)],
                      dtype=np.uint64)
    assert np.array_equal(hashes, rhash)
    # the escaped {lit} of ~10 % of the strings is live after the unescape and resolves to LIT
    assert 0.08 < ob.count(b"LIT") / n < 0.12
    N.lib().ie_table_free(table)


def test_unescape_command_tmp_too_small_reports_capacity():
    """a tmp buffer smaller than the unescaped strings. The command must read
    nothing past it (the unescape step writes all offsets as 0 on overflow) and ie_exec_sync must
    report IE_ERR_CAPACITY; a tmp of the right size then gives the oracle's results."""
    h, kvp, nkv = _synth(4)
    table = _table_from_kv(kvp, nkv)
    x = N.Exec(0)
    n = 50_000
    buf, offs = _host_strings(h, 0, n)
    d_bytes = N.DeviceBuffer.from_numpy(x, buf)
    d_off = N.DeviceBuffer.from_numpy(x, offs)
    r = _device_run(x, table, d_bytes, d_off, n)
    tmp = DevResult(x, n, 4096)  # far too small
    out = DevResult(x, n, 2 * r.total() + 4096)
    N.check(N.lib().ie_unescape_cmd_device(x.h, table, None, r.bytes.ptr, r.off.ptr, n, r.status.ptr,
                                           ctypes.byref(tmp.out), ctypes.byref(out.out)), "ie_unescape_cmd_device")
    assert N.lib().ie_exec_sync(x.h) == -6  # IE_ERR_CAPACITY
    assert tmp.total() > 4096
    assert int(np.count_nonzero(tmp.off.to_numpy(np.uint64, n + 1))) == 0
    _, u = _unescape_cmd(x, table, r, n, r.total() + 4096)
    ref = O.Oracle.from_kv(ctypes.cast(kvp, ctypes.c_void_p), nkv, "py", clock=CLOCK)
    rst = np.zeros(n, np.uint8)
    ref.run_batch(buf, offs, n, 8, rst, None, None, None, unescape_cmd=True)
    assert np.array_equal(u.status.to_numpy(np.uint8, n), rst)
    N.lib().ie_table_free(table)


def test_full_size_config4_properties():
    """Config 4 at its per-GPU size (100M strings sharded 8 ways = 12.5M; this is rank 3's shard):
    mixed-depth chains, escapes, brace-bearing values and misses, then the `unescape` command
    (recursive_unescape, then recursive_interpolate: py:1660-1667) over the outputs. Properties:
    statuses are OK_STR or E_INTERP only, misses ~1 %, the unescaped text is the resolved text with
    every backslash-brace pair's backslash removed, the command's outputs carry no brace (the
    un-escaped {lit} resolved again), idempotence of the second resolve; plus a sampled oracle
    check of both passes."""
    h, kvp, nkv = _synth(4)
    table = _table_from_kv(kvp, nkv)
    x = N.Exec(0)
    n = 12_500_000
    first = 3 * n
    d_off, d_bytes, in_total = _device_strings(x, h, first, n)
    r = _device_run(x, table, d_bytes, d_off, n)
    tot = r.total()
    st = r.status.to_numpy(np.uint8, n)
    names = N.STATUS_NAMES
    ok = st == names.index("OK_STR")
    miss = st == names.index("E_INTERP")
    counts = {names[k]: int(c) for k, c in enumerate(np.bincount(st, minlength=len(names))[:len(names)]) if c}
    assert int(np.count_nonzero(ok | miss)) == n, (counts, np.flatnonzero(~(ok | miss))[:10])
    assert 0.005 < np.count_nonzero(miss) / n < 0.015
    oo = r.off.to_numpy(np.uint64, n + 1)
    assert int(oo[-1]) == tot and np.all(np.diff(oo.astype(np.int64)) >= 0)
    ob = r.bytes.to_numpy(np.uint8, tot)
    tmp, u = _unescape_cmd(x, table, r, n, tot + 4096)
    utot = tmp.total()
    ub = tmp.bytes.to_numpy(np.uint8, utot)
    n_esc = int(np.count_nonzero((ob[:-1] == ord("\\")) & (ob[1:] == ord("{"))))
    n_esc += int(np.count_nonzero((ob[:-1] == ord("\\")) & (ob[1:] == ord("}"))))
    assert n_esc > 0 and utot == tot - n_esc
    assert int(np.count_nonzero(ub == ord("\\"))) == 0
    ust = u.status.to_numpy(np.uint8, n)
    assert np.array_equal(ust, st)  # the un-escaped {lit} always resolves; failures carry through
    uo = u.off.to_numpy(np.uint64, n + 1)
    ftot = u.total()
    fb = u.bytes.to_numpy(np.uint8, ftot)
    assert int(np.count_nonzero(fb == ord("{"))) == 0 and int(np.count_nonzero(fb == ord("}"))) == 0
    rng = np.random.default_rng(4)
    ref = O.Oracle.from_kv(ctypes.cast(kvp, ctypes.c_void_p), nkv, "py", clock=CLOCK)
    for i in np.sort(rng.choice(n, 500, replace=False)):
        b, o = _host_strings(h, first + int(i), 1)
        rs, rout, _ = ref.interpolate(b[:int(o[1])].tobytes())
        assert rs == names[st[i]]
        if rs == "OK_STR":
            assert ob[int(oo[i]):int(oo[i + 1])].tobytes().decode("utf-8") == rout
            rs2, rout2, _ = ref.interpolate(rout.replace("\\{", "{").replace("\\}", "}").encode())
            assert rs2 == "OK_STR"
            assert fb[int(uo[i]):int(uo[i + 1])].tobytes().decode("utf-8") == rout2
    N.lib().ie_table_free(table)


def test_device_scratch_autogrow_and_caller_sized():
    """ie_interpolate_device grows the literal path's scratch pool to the batch's demand and re-runs
    (no IE_E_OVERFLOW from capacity); a pool sized by the caller (ie_exec_set_scratch) keeps the
    call asynchronous and reports the strings that did not fit as IE_E_OVERFLOW. The table keeps
    its raw brace-bearing values (IE_NO_PRERESOLVE) so config 4's 2 % take the literal path."""
    h, kvp, nkv = _synth(4)
    os.environ["IE_NO_PRERESOLVE"] = "1"
    try:
        table = _table_from_kv(kvp, nkv)
    finally:
        del os.environ["IE_NO_PRERESOLVE"]
    n = 300_000
    over = N.STATUS_NAMES.index("E_OVERFLOW")
    x = N.Exec(0)
    d_off, d_bytes, _ = _device_strings(x, h, 0, n)
    N.check(N.lib().ie_exec_set_scratch(x.h, 1 << 20), "scratch")
    small = _device_run(x, table, d_bytes, d_off, n).status.to_numpy(np.uint8, n)
    assert int(np.count_nonzero(small == over)) > 0
    y = N.Exec(0)
    d_off2, d_bytes2, _ = _device_strings(y, h, 0, n)
    full = _device_run(y, table, d_bytes2, d_off2, n).status.to_numpy(np.uint8, n)
    assert int(np.count_nonzero(full == over)) == 0
    assert np.array_equal(full[small != over], small[small != over])
    N.lib().ie_table_free(table)


@pytest.mark.parametrize("op", ["ie_unescape_device", "ie_escape_device"])
def test_escape_kernels_on_a_ragged_batch(op):
    """recursive_unescape / recursive_escape on strings (py:1436-1460) over a ragged batch: empty
    strings, short strings, strings longer than an LDS tile, backslash runs next to braces."""
    rng = random.Random(5)
    alpha = ["a", "{", "}", "\\", "\\{", "\\}", "é", "😀", " "]
    strs = []
    for k in range(60_000):
        r = rng.random()
        n = 0 if r < 0.05 else rng.randint(1, 20) if r < 0.9 else rng.randint(200, 3000)
        if k % 9000 == 0:
            n = 40_000  # a tile beyond the LDS stage
        strs.append("".join(rng.choice(alpha) for _ in range(n)))
    enc = [t.encode() for t in strs]
    offs = np.zeros(len(enc) + 1, np.uint64)
    offs[1:] = np.cumsum([len(b) for b in enc])
    buf = np.frombuffer(b"".join(enc) + bytes(16), np.uint8)
    n = len(enc)
    x = N.Exec(0)
    d_b = N.DeviceBuffer.from_numpy(x, buf)
    d_o = N.DeviceBuffer.from_numpy(x, offs)
    res = DevResult(x, n, 2 * buf.size + 4096)
    N.check(getattr(N.lib(), op)(x.h, d_b.ptr, d_o.ptr, n, ctypes.byref(res.out)), op)
    x.sync()
    o1 = res.off.to_numpy(np.uint64, n + 1)
    b1 = res.bytes.to_numpy(np.uint8, res.total()).tobytes()
    assert int(np.count_nonzero(res.status.to_numpy(np.uint8, n))) == 0
    for k, t in enumerate(strs):
        want = (t.replace("\\{", "{").replace("\\}", "}") if op == "ie_unescape_device"
                else t.replace("{", "\\{").replace("}", "\\}"))
        assert b1[int(o1[k]):int(o1[k + 1])].decode() == want, k


def test_fail_commit_is_adopted_after_a_batch_with_misses(monkeypatch):
    """Adaptive variant choice: an exec starts with chain failures on the exact evaluator, switches
    once an earlier batch showed chain failures, and switches back after a batch without any;
    results are identical throughout."""
    monkeypatch.delenv("IE_FAIL_COMMIT", raising=False)
    h, kvp, nkv = _synth(4)
    table = _table_from_kv(kvp, nkv)
    x = N.Exec(0)
    n = 200_000
    d_off, d_bytes, _ = _device_strings(x, h, 0, n)
    runs = []
    for _ in range(3):
        x.set_timing(True)
        r = _device_run(x, table, d_bytes, d_off, n)
        tm = x.timing()
        x.set_timing(False)
        runs.append((int(tm.n_exact), r.off.to_numpy(np.uint64, n + 1), r.bytes.to_numpy(np.uint8, r.total()),
                     r.status.to_numpy(np.uint8, n)))
    assert runs[0][0] > n // 1024  # misses went to the exact evaluator
    assert runs[2][0] == 0  # ... and are committed by the chain evaluator later
    for k in (1, 2):
        assert np.array_equal(runs[k][1], runs[0][1]) and np.array_equal(runs[k][2], runs[0][2])
        assert np.array_equal(runs[k][3], runs[0][3])
    # a stream without chain failures (config 3) switches back to the lean variant
    h3, kvp3, nkv3 = _synth(3)
    t3 = _table_from_kv(kvp3, nkv3)
    d_off3, d_bytes3, _ = _device_strings(x, h3, 0, n)
    fails = []
    for _ in range(3):
        x.set_timing(True)
        _device_run(x, t3, d_bytes3, d_off3, n)
        fails.append(int(x.timing().n_chain_fail))
        x.set_timing(False)
    assert fails == [0, 0, 0]
    N.lib().ie_table_free(t3)
    N.lib().ie_table_free(table)


def test_device_api_capacity_contract():
    """bytes_cap too small: offsets/status are valid, *total reports the need, bytes untouched."""
    t = PKG.InsertsTable({"a": "A" * 50}, clock=CLOCK)
    x = N.Exec(0)
    strings = ["x{a}y"] * 600
    blob, offs = N.pack(strings)
    d_bytes = N.DeviceBuffer.from_numpy(x, np.frombuffer(blob, np.uint8))
    d_off = N.DeviceBuffer.from_numpy(x, offs)
    r = _device_run(x, t.h, d_bytes, d_off, len(strings), cap=100)
    total = r.total()
    assert total == 52 * 600
    assert int(r.off.to_numpy(np.uint64, 601)[-1]) == total
    assert int(np.count_nonzero(r.status.to_numpy(np.uint8, 600))) == 0
    r = _device_run(x, t.h, d_bytes, d_off, len(strings), cap=total)
    assert r.bytes.to_numpy(np.uint8, total).tobytes() == ("x" + "A" * 50 + "y").encode() * 600


def test_device_escape_entry_points():
    x = N.Exec(0)
    strings = ["a{b}c", "\\{x\\}", "", "{{}}"] * 300
    blob, offs = N.pack(strings)
    d_bytes = N.DeviceBuffer.from_numpy(x, np.frombuffer(blob, np.uint8))
    d_off = N.DeviceBuffer.from_numpy(x, offs)
    for fn, unesc in ((N.lib().ie_escape_device, False), (N.lib().ie_unescape_device, True)):
        r = DevResult(x, len(strings), 4 * len(blob) + 64)
        N.check(fn(x.h, d_bytes.ptr, d_off.ptr, len(strings), ctypes.byref(r.out)), "escape")
        x.sync()
        oo = r.off.to_numpy(np.uint64, len(strings) + 1)
        ob = r.bytes.to_numpy(np.uint8, r.total()).tobytes()
        got = [ob[int(oo[i]):int(oo[i + 1])].decode() for i in range(len(strings))]
        assert got == [O.escape(s, unescape=unesc) for s in strings]


# ------------------------------------------------------------------------------------------
# escape / unescape (py:1436-1460)
# ------------------------------------------------------------------------------------------
def test_escape_unescape_golden():
    rows = load_golden("escape_py.jsonl")
    ss = [r["s"] for r in rows]
    assert PKG.recursive_escape(ss) == [r["esc"] for r in rows]
    assert PKG.recursive_unescape(ss) == [r["unesc"] for r in rows]


def test_escape_roundtrip_property():
    rng = random.Random(11)
    ss = ["".join(rng.choice(["{", "}", "\\", "a", "é", "\\{", "."]) for _ in range(rng.randint(0, 300)))
          for _ in range(5000)]
    assert PKG.recursive_unescape(PKG.recursive_escape(ss)) == ss


# ------------------------------------------------------------------------------------------
# the mirror of the reference module surface
# ------------------------------------------------------------------------------------------
def test_mirror_surface_raises_like_the_reference():
    ins = {"name": "tom", "i": 3, "question-3": "Why?", "L": ["x", "y"], "f": 1.5, "d": {"k": 1}}
    assert PKG.interpolate_inserts(ins, "My name is {name}.") == "My name is tom."
    assert PKG.interpolate_inserts(ins, "{question-{i}}") == "Why?"
    assert PKG.interpolate_inserts(ins, "{L}") is ins["L"]
    with pytest.raises(PKG.InterpolationException):
        PKG.interpolate_inserts(ins, "x{nope}")
    with pytest.raises(AssertionError):
        PKG.interpolate_inserts(ins, "x{f}")
    with pytest.raises(AssertionError):
        PKG.interpolate_inserts(ins, "a{b")
    with pytest.raises(TypeError):
        PKG.interpolate_inserts(ins, "{{L}}")
    ins["name"] = "ann"  # the cached device table notices the change
    assert PKG.interpolate_inserts(ins, "{name}") == "ann"
    ins["L"].append("z")
    assert PKG.interpolate_inserts(ins, "x{L}") == "x['x', 'y', 'z']"


def test_recursive_interpolate_golden():
    rows = load_golden("recursive_py.jsonl")
    table = rows[0]["table"]
    for row in rows[1:]:
        if "x" in row:
            if row["st"] == "OK":
                assert PKG.recursive_interpolate(table, row["x"]) == row["out"], row
            else:
                exc = PKG.InterpolationException if row["st"] == "E_INTERP" else AssertionError
                with pytest.raises(exc):
                    PKG.recursive_interpolate(table, row["x"])
        else:
            assert PKG.recursive_escape(row["esc_in"]) == row["esc"]
            assert PKG.recursive_unescape(row["esc_in"]) == row["unesc"]


# ------------------------------------------------------------------------------------------
# table sets: many inserts dicts in one device table, a table id per string (config 5, §8b)
# ------------------------------------------------------------------------------------------
@pytest.mark.parametrize("dialect", ["py", "rs"])
def test_table_set_matches_per_table_oracle(dialect, fail_commit):
    """Every string resolves against its own dict: same keys with different values in different
    tables, brace-bearing values pre-resolved against their own table, clock entries per table."""
    rng = random.Random(99)
    tables = [_rand_table(rng, rng.randint(5, 40), brace_values=(k % 2 == 0)) for k in range(37)]
    tables[3] = {}  # an empty dict in the set
    tables[5]["k1"] = "{HH:MM}-{k2}"
    items = []
    for _ in range(6000):
        t = rng.randrange(len(tables))
        items.append((t, _rand_string(rng, 40)))
    items += [(t, "{HH:MM:SS}") for t in range(len(tables))] + [(5, "x{k1}")]
    tset = PKG.InsertsTableSet(tables, dialect=dialect, clock=CLOCK)
    got = tset.run([s for _, s in items], [t for t, _ in items])
    oracles = [O.Oracle(tb, dialect, clock=CLOCK) for tb in tables]
    bad = []
    for (t, s), (st, payload) in zip(items, got):
        rst, rout, rvid = oracles[t].interpolate(s)
        name = N.STATUS_NAMES[st]
        ok = name == rst
        if ok and rst == "OK_STR":
            ok = payload == rout
        if ok and rst == "OK_VALUE":  # value ids index the concatenated kv list of the set
            ok = payload == (rvid if rvid >= 0xFFFFFFF0 else rvid + tset.starts[t])
        if not ok:
            bad.append((t, s, name, payload, rst, rout, rvid))
    assert not bad, (len(bad), bad[:4])


def test_table_set_device_ids_out_of_range_find_nothing():
    """Device API: an id beyond the set reports missing keys (no memory is indexed by the id);
    the host API refuses such ids."""
    tset = PKG.InsertsTableSet([{"a": "A"}, {"a": "B"}], clock=CLOCK)
    x = N.Exec(0)
    strings = ["x{a}", "x{a}", "x{a}", "plain"]
    ids = np.array([0, 1, 7, 7], np.uint32)
    blob, offs = N.pack(strings)
    d_bytes = N.DeviceBuffer.from_numpy(x, np.frombuffer(blob, np.uint8))
    d_off = N.DeviceBuffer.from_numpy(x, offs)
    d_ids = N.DeviceBuffer.from_numpy(x, ids)
    r = DevResult(x, len(strings), 256)
    N.check(N.lib().ie_interpolate_device_ids(x.h, tset.h, d_ids.ptr, d_bytes.ptr, d_off.ptr, len(strings),
                                              ctypes.byref(r.out)), "ids")
    x.sync()
    st = [N.STATUS_NAMES[v] for v in r.status.to_numpy(np.uint8, 4)]
    assert st == ["OK_STR", "OK_STR", "E_INTERP", "OK_STR"]
    oo = r.off.to_numpy(np.uint64, 5)
    ob = r.bytes.to_numpy(np.uint8, r.total()).tobytes()
    assert [ob[int(oo[i]):int(oo[i + 1])] for i in (0, 1, 3)] == [b"xA", b"xB", b"plain"]
    with pytest.raises(RuntimeError):
        tset.run(strings, [0, 1, 7, 7])


def test_table_clock_rewritten_in_place():
    t = PKG.InsertsTable({"k": "v", "w": "{k}"}, clock=(1, 2, 3))
    assert t.results(["{HH:MM}", "x{HH:MM:SS}", "{w}"]) == ["01:02", "x01:02:03", "{k}"]
    assert t.set_clock((23, 59, 58))
    assert t.results(["{HH:MM}", "x{HH:MM:SS}", "x{w}"]) == ["23:59", "x23:59:58", "xv"]



def test_clock_read_through_values_follows_set_clock():
    """values that read the clock, directly or through a nested key ('{{a}}' with
    a = 'HH:MM', '{HH:{m}}'), are not pre-resolved at build, so a spliced lookup after set_clock
    sees the new time like the reference's datetime.now() (py:433-436); clock-free brace values
    still are pre-resolved. Checked against the oracle under the new clock."""
    table = {"w": "at {HH:MM}", "a": "HH:MM", "v": "<{{a}}>", "m": "MM:SS", "u": "[{HH:{m}}]", "k": "K",
             "plain": "p{k}q", "x": "{w}{plain}"}
    strings = ["x{w}", "x{v}", "x{u}", "-{x}", "x{plain}", "a{HH:MM}", "x{HH:MM:SS}"]
    t = PKG.InsertsTable(table, clock=(1, 2, 3))
    ref = O.Oracle(table, "py", clock=(1, 2, 3))
    assert t.results(strings) == [ref.interpolate(s)[1] for s in strings]
    for clock in [(4, 5, 6), (23, 59, 58)]:
        assert t.set_clock(clock)
        ref = O.Oracle(table, "py", clock=clock)
        assert t.results(strings) == [ref.interpolate(s)[1] for s in strings]
    assert t.results(["x{u}"]) == ["x[23:59:58]"]


def test_mirror_table_cache_versioned_and_bounded():
    ins = PKG.VersionedInserts(name="tom", n=1)
    assert PKG.interpolate_inserts(ins, "hi {name}") == "hi tom"
    t1 = PKG.interpolation_engine.table_for(ins)
    assert PKG.interpolation_engine.table_for(ins) is t1  # unchanged: no rebuild
    ins["name"] = "ann"
    assert PKG.interpolate_inserts(ins, "hi {name}") == "hi ann"
    dicts = [{"k": str(j)} for j in range(20)]
    for d in dicts:
        assert PKG.interpolate_inserts(d, "{k}") == d["k"]
    assert len(PKG.interpolation_engine._cache) <= PKG.interpolation_engine._CACHE_SIZE


def test_mirror_refresh_from_logged_keys_matches_oracle():
    """A scalar caller's dict mutated between calls (py:470-471 stores and `del`, a bulk update,
    an in-place list change announced with bump(), a store of the same object): each
    interpolate_inserts refreshes the cached table from VersionedInserts' log of stored keys (or a
    whole-dict comparison where the log does not reach) and must equal the oracle on the live dict."""
    rng = random.Random(5)
    keys = ["k%d" % j for j in range(24)]
    ins = PKG.VersionedInserts({k: "v" + k for k in keys})
    ins["L"] = ["a", 1]
    ins["nest"] = "<{k3}>"
    strings = ["{k0}|{k5}|{nest}", "x{k%d}y" % 7, "{{k1}}", "L={L}", "n{nest}{k23}"]
    ie = PKG.interpolation_engine
    for step in range(60):
        r = rng.random()
        if r < 0.45:
            ins[rng.choice(keys)] = rng.choice(["s%d" % step, "{k2}", "", "tail {k4}.", "k1"])
        elif r < 0.55:
            k = rng.choice(keys[8:])
            if k in ins:
                del ins[k]
        elif r < 0.65:
            ins.update({rng.choice(keys): "u%d" % step, "new%d" % step: "n"})
        elif r < 0.75:
            ins["L"].append(step)
            ins.bump()
        elif r < 0.85:
            k = rng.choice(keys[:8])
            ins[k] = ins[k]  # the same object again
        else:
            ins["k%d" % rng.randrange(24)] = ["x", step]
        ref = O.Oracle({k: v for k, v in ins.items()}, "py", clock=CLOCK)
        for s in strings:
            st, out, _ = ref.interpolate(s)
            if st == "OK_STR":
                assert ie.interpolate_inserts(ins, s) == out, (step, s)
            elif st == "OK_VALUE":
                assert ie.interpolate_inserts(ins, s) is ins[s[1:-1]], (step, s)
            else:
                with pytest.raises(Exception):
                    ie.interpolate_inserts(ins, s)
    ie.table_for(ins)  # (the cached table still follows the dict)


def test_interpolate_states_batch():
    states = [{"scenario": "s%d" % j, "stage": "first", "L": [j]} for j in range(50)]
    items = [(j % 50, c) for j, c in enumerate(["{scenario}", "x{stage}|{scenario}", "{L}", "{nope}"] * 50)]
    res = PKG.interpolate_states(states, items)
    for (j, c), r in zip(items, res):
        if c == "{nope}":
            assert isinstance(r, PKG.InterpolationException)
        elif c == "{L}":
            assert r is states[j]["L"]
        else:
            assert r == c.replace("{scenario}", states[j]["scenario"]).replace("{stage}", "first")


def test_ingestion_and_display_sites():
    """SURVEY §8f-3 on the device kernels: user_input escaping (py:1564-1568), ARGn seeding
    (py:2343-2349) and the print command's unescape (py:1669-1673), against the oracle's byte
    maps; a non-str print text raises AttributeError as the reference's .replace does."""
    rng = random.Random(21)
    texts = ["", "{", "}", "\\{x\\}", "a{b}c", "é{😀}", "{{}}", "\\\\{"]
    texts += ["".join(rng.choice("ab{}\\\\ é") for _ in range(rng.randrange(0, 40))) for _ in range(300)]
    assert PKG.ingest_user_inputs(texts) == [O.escape(t) for t in texts]
    assert PKG.ingest_user_input("say {hi}") == "say \\{hi\\}"
    assert PKG.ingest_args(["x{y}", "z"]) == {"ARG1": "x\\{y\\}", "ARG2": "z"}
    assert PKG.display_texts(texts) == [O.escape(t, unescape=True) for t in texts]
    with pytest.raises(AttributeError):
        PKG.display_text(5)


def test_rust_dialect_hand_derived_vectors():
    """The hand-derived interp.rs vectors of test_oracle_golden.py on the device (rs dialect)."""
    from tests.test_oracle_golden import test_oracle_rust_dialect_restated as T
    cases = [m.args[1] for m in T.pytestmark if m.name == "parametrize"][0]
    t = {"a": "A", "L": ["x", "y"], "f": 1.5, "k": "K", "open": "}{", "n": 5, "5": "five", "t": True,
         "nested": ["p", [1, 2], {"z": 1}], "none": None, "obj": {"b": 2}, "q-5": "Q5", "i": 5, "neg": -3,
         "two": 2.0, "bs": "q\\", "e": "", "big": 12345678901234567890}
    got, _ = run_product(t, [s for s, _ in cases], "rs")
    for (s, want), (st, payload) in zip(cases, got):
        assert N.STATUS_NAMES[st] == want[0], (s, N.STATUS_NAMES[st], want)
        if want[1] is not None and want[0] == "OK_STR":
            assert payload == want[1], (s, payload)
        if want[1] is not None and want[0] == "OK_VALUE":
            assert list(t)[payload] == want[1], (s, payload)


@pytest.mark.gpu
def test_tile_option_is_validated_and_keeps_results():
    """IE_OPT_TILE takes 0, 256 or 512 and nothing else; every size gives the same bytes."""
    x = N.Exec(0)
    with pytest.raises(RuntimeError):
        x.set_option(N.OPT_TILE, 384)
    table = {"k%d" % i: "v%d" % i for i in range(50)}
    strings = ["a{k%d}b{k%d}" % (i % 50, (7 * i) % 50) for i in range(3000)] + ["plain %d" % i for i in range(3000)]
    ie = PKG.interpolation_engine
    got = []
    for tile in (256, 512, 0):
        ie.get_exec(0).set_option(N.OPT_TILE, tile)
        got.append(run_product(table, strings)[0])
    ie.get_exec(0).set_option(N.OPT_TILE, 0)
    assert got[0] == got[1] == got[2]



# ------------------------------------------------------------------------------------------
# the `unescape` command's recursion into whole-string results (py:1463-1464)
# ------------------------------------------------------------------------------------------
def test_unescape_command_device_statuses_match_oracle():
    """ie_unescape_cmd_device on the reference-generated items: statuses (including IE_RECURSE for
    whole-string items whose result recursive_interpolate re-enters), bytes and value ids equal the
    oracle's command (ieo_run_batch mode 2)."""
    g = load_golden("unescape_cmd_py.json")
    table, rows = g["table"], g["rows"]
    strings = [r["s"] for r in rows]
    t = PKG.InsertsTable(table, clock=CLOCK)
    x = N.Exec(0)
    blob, offs = N.pack(strings)
    n = len(strings)
    d_bytes = N.DeviceBuffer.from_numpy(x, np.frombuffer(blob + bytes(16), np.uint8))
    d_off = N.DeviceBuffer.from_numpy(x, offs)
    tmp, out = DevResult(x, n, len(blob) + 4096), DevResult(x, n, 64 * len(blob) + (1 << 20))
    N.check(N.lib().ie_unescape_cmd_device(x.h, t.h, None, d_bytes.ptr, d_off.ptr, n, None, ctypes.byref(tmp.out),
                                           ctypes.byref(out.out)), "ie_unescape_cmd_device")
    x.sync()
    st = out.status.to_numpy(np.uint8, n)
    oo = out.off.to_numpy(np.uint64, n + 1)
    ob = out.bytes.to_numpy(np.uint8, out.total()).tobytes()
    vid = out.vid.to_numpy(np.uint32, n)
    ref = O.Oracle(table, "py", clock=CLOCK)
    buf = np.frombuffer(blob + b"\0", np.uint8)
    rst, rlen, rhash, rvid = np.zeros(n, np.uint8), np.zeros(n, np.uint64), np.zeros(n, np.uint64), np.zeros(n, np.uint32)
    ref.run_batch(buf, offs, n, 4, rst, rlen, rhash, rvid, command_only=True)
    # a runaway item (self-referential inserts) outgrows the device call's single-pass budget:
    # IE_E_OVERFLOW where the oracle runs on to its cap (the host batch API re-runs those in max
    # mode; the device entry reports them, include/ie_amd.h)
    over = (st == N.E_OVERFLOW) & (rst == N.DIVERGED)
    st = np.where(over, rst, st)
    assert np.array_equal(st, rst), [(strings[i], st[i], rst[i]) for i in np.flatnonzero(st != rst)[:8]]
    ok = st == N.OK_STR
    assert np.array_equal(np.diff(oo.astype(np.int64))[ok], rlen.astype(np.int64)[ok])
    for i in np.flatnonzero(ok):
        assert O.fnv1a(ob[int(oo[i]):int(oo[i + 1])]) == int(rhash[i]), strings[i]
    typed = (st == N.OK_VALUE) | (st == N.RECURSE)
    assert np.array_equal(vid[typed], rvid[typed])
    assert int(np.count_nonzero(st == N.RECURSE)) > 20
    t.close()


def test_unescape_command_mirror_matches_reference(monkeypatch):
    """The mirror's unescape_command (recursive_unescape, then recursive_interpolate, both on the
    device) reproduces the reference's result for every item, including the recursion. The clock
    is the generator's (12:34:56)."""
    import datetime as real_dt
    import types

    class _Fixed(real_dt.datetime):
        @classmethod
        def now(cls, tz=None):
            return real_dt.datetime(2026, 1, 1, *CLOCK)

    monkeypatch.setattr(PKG.interpolation_engine, "_dt", types.SimpleNamespace(datetime=_Fixed))
    g = load_golden("unescape_cmd_py.json")
    table, rows = g["table"], g["rows"]
    exc = {"E_INTERP": PKG.InterpolationException, "E_ASSERT_BRACES": AssertionError,
           "E_ASSERT_TYPE": AssertionError, "E_UNHASHABLE": TypeError, "DIVERGED": RecursionError}
    bad = []
    for r in rows:
        try:
            got = PKG.unescape_command(table, r["s"])
        except Exception as e:  # noqa: BLE001 — the class is what is compared
            if r["st"] not in exc or not isinstance(e, exc[r["st"]]):
                bad.append((r, repr(e)))
            continue
        want = r.get("out", r.get("value"))
        if r["st"] not in ("OK_STR", "OK_VALUE") or got != want or type(got) != type(want):
            bad.append((r, got))
    assert not bad, (len(bad), bad[:5])


# ------------------------------------------------------------------------------------------
# the fused unescape command on a views batch (ie_unescape_cmd_device_views)
# ------------------------------------------------------------------------------------------
def _cmd_views(x, table, strings, ids=None, views_input=False, seed=0):
    """The command through the fused views entry; (status, [bytes], value ids) per string. A views
    input places the strings in a shuffled order with a brace or backslash between them (bytes
    that belong to no string)."""
    n = len(strings)
    enc = [s.encode("utf-8") for s in strings]
    d_len = None
    if views_input:
        rng = random.Random(seed)
        order = list(range(n))
        rng.shuffle(order)
        parts, offs, pos = [], np.zeros(n, np.uint64), 0
        for i in order:
            gap = rng.choice([b"{", b"}", b"\\", b"", b"x{"])
            parts += [gap, enc[i]]
            offs[i] = pos + len(gap)
            pos += len(gap) + len(enc[i])
        blob = b"".join(parts)
        lens = np.array([len(e) for e in enc], np.uint32)
        d_len = N.DeviceBuffer.from_numpy(x, lens)
    else:
        blob, offs = N.pack(strings)
    d_bytes = N.DeviceBuffer.from_numpy(x, np.frombuffer(blob + bytes(16), np.uint8))
    d_off = N.DeviceBuffer.from_numpy(x, offs)
    cap = 64 * len(blob) + (1 << 20)
    out = N.DeviceBuffer(x, cap)
    o_off, o_len = N.DeviceBuffer(x, 8 * n + 8), N.DeviceBuffer(x, 4 * n + 4)
    o_st, o_vid, o_tot = N.DeviceBuffer(x, n + 1), N.DeviceBuffer(x, 4 * n + 4), N.DeviceBuffer(x, 8)
    v = N.DevViews(out.ptr, cap, o_off.ptr, o_len.ptr, o_st.ptr, o_vid.ptr, o_tot.ptr)
    N.check(N.lib().ie_unescape_cmd_device_views(x.h, table, ids, d_bytes.ptr, d_off.ptr,
                                                 d_len.ptr if d_len else None, n, None, ctypes.byref(v)),
            "ie_unescape_cmd_device_views")
    x.sync()
    tot = int(o_tot.to_numpy(np.uint64, 1)[0])
    st = o_st.to_numpy(np.uint8, n)
    starts, ln = o_off.to_numpy(np.uint64, n), o_len.to_numpy(np.uint32, n)
    ob = out.to_numpy(np.uint8, tot).tobytes()
    assert int(ln[st == N.OK_STR].sum()) == tot  # the payload is the OK strings, gap-free
    res = [ob[int(starts[i]):int(starts[i]) + int(ln[i])] if st[i] == N.OK_STR else None for i in range(n)]
    return st, res, o_vid.to_numpy(np.uint32, n)


def _cmd_oracle(ref, strings):
    blob, offs = N.pack(strings)
    n = len(strings)
    buf = np.frombuffer(blob + b"\0", np.uint8)
    rst, rlen, rhash, rvid = np.zeros(n, np.uint8), np.zeros(n, np.uint64), np.zeros(n, np.uint64), np.zeros(n, np.uint32)
    ref.run_batch(buf, offs, n, 4, rst, rlen, rhash, rvid, command_only=True)
    return rst, rlen, rhash, rvid


def _assert_cmd_equal(strings, got, want, allow_overflow=False):
    st, res, vid = got
    rst, rlen, rhash, rvid = want
    if allow_overflow:  # the runaway items, as test_unescape_command_device_statuses_match_oracle
        st = np.where((st == N.E_OVERFLOW) & (rst == N.DIVERGED), rst, st)
    bad = [(strings[i][:60], int(st[i]), int(rst[i])) for i in np.flatnonzero(st != rst)[:8]]
    assert not bad, bad
    for i in np.flatnonzero(st == N.OK_STR):
        assert len(res[i]) == int(rlen[i]) and O.fnv1a(res[i]) == int(rhash[i]), strings[i][:80]
    typed = (st == N.OK_VALUE) | (st == N.RECURSE)
    assert np.array_equal(vid[typed], rvid[typed])


@pytest.mark.parametrize("views_input", [False, True], ids=["packed-in", "views-in"])
def test_unescape_command_views_golden(views_input, fail_commit):
    """The reference-generated command items through the fused views entry."""
    g = load_golden("unescape_cmd_py.json")
    strings = [r["s"] for r in g["rows"]]
    t = PKG.InsertsTable(g["table"], clock=CLOCK)
    x = N.Exec(0)  # (the fixture's environment: fail-commit variant)
    got = _cmd_views(x, t.h, strings, views_input=views_input)
    _assert_cmd_equal(strings, got, _cmd_oracle(O.Oracle(g["table"], "py", clock=CLOCK), strings), True)
    assert int(np.count_nonzero(got[0] == N.RECURSE)) > 20
    t.close()


@pytest.mark.parametrize("dialect", ["py", "rs"])
@pytest.mark.parametrize("views_input", [False, True], ids=["packed-in", "views-in"])
def test_unescape_command_views_edges(dialect, views_input):
    """Escapes at string boundaries (a '\\\\' that ends a string before the next one's brace keeps
    its backslash), backslash runs, multibyte text around escapes, empty strings, strings longer
    than the LDS stage (the deferred pass) and random escape-bearing strings, both dialects."""
    rng = random.Random(5)
    table = _rand_table(rng, 50, True)
    table.update({"lit": "LIT", "a}b": "AB", "a{b": "AB2", "{": "BR", "k\\": "KB"})
    strings = ["x\\", "{k1}", "y\\", "}z", "\\", "{", "\\\\{lit\\}", "\\{lit\\}", "é\\{lit\\}😀", "", "\\{\\{lit\\}\\}",
               "{a\\}b}", "{a\\{b}", "\\{\\}", "{\\{}", "a\\\\\\}b", "{k\\}", "k\\", "\\}{k2}", "{k3}\\"]
    # past the stage, within the device entry's single-pass budget of 2048 substitutions (beyond
    # it the device entry reports IE_E_OVERFLOW and the batch API re-runs: include/ie_amd.h)
    strings += ["p\\{lit\\}" * 2000 + "é" * 3000, "{k1}" * 1500 + "\\{lit\\}" + "z" * 15000,
                "\\" * 20000 + "{" + "x" * 100 + "}", "x" * 18000 + "\\{lit\\}\\", "{k2}y\\{lit\\}" * 800]
    strings += [_rand_string(rng, 50, long=rng.random() < 0.2) for _ in range(6000)]
    t = PKG.InsertsTable(table, dialect=dialect, clock=CLOCK)
    x = N.Exec(0)
    got = _cmd_views(x, t.h, strings, views_input=views_input, seed=3)
    _assert_cmd_equal(strings, got, _cmd_oracle(O.Oracle(table, dialect, clock=CLOCK), strings), True)
    t.close()


def test_unescape_command_views_table_set():
    """The fused command with a table-id batch (one inserts dict per state)."""
    rng = random.Random(9)
    dicts = [dict(_rand_table(rng, 30, True), lit="L%d" % j) for j in range(5)]
    strings = [_rand_string(rng, 30) + "\\{lit\\}" for _ in range(4000)]
    ids = np.array([rng.randrange(5) for _ in strings], np.uint32)
    tset = PKG.InsertsTableSet(dicts, clock=CLOCK)
    x = N.Exec(0)
    d_ids = N.DeviceBuffer.from_numpy(x, ids)
    st, res, vid = _cmd_views(x, tset.h, strings, ids=d_ids.ptr, views_input=True)
    for j in range(5):
        sel = np.flatnonzero(ids == j)
        sub = [strings[i] for i in sel]
        rst, rlen, rhash, rvid = _cmd_oracle(O.Oracle(dicts[j], "py", clock=CLOCK), sub)
        got = (st[sel], [res[i] for i in sel], vid[sel].astype(np.int64) - tset.starts[j])
        want = (rst, rlen, rhash, rvid.astype(np.int64))
        _assert_cmd_equal(sub, got, want, True)
    tset.close()


def test_one_string_calls_without_the_emit_kernel():
    """A one-tile views call runs k_resolve alone (it writes the total); a tile whose output it must
    defer (past the LDS stage: a long value, a long string) comes back with the deferred count and
    the call runs again on the generic path. Every case equals the oracle, through run1 (the scalar
    interpolate_inserts path) and through a batch of the same strings."""
    x = PKG.interpolation_engine.get_exec(0)
    x.set_option(N.OPT_VIEWS, 1)
    try:
        table = {"k": "v" * 70000, "s": "short", "n": "{s}-{s}", "m": "é" * 30000, "e": ""}
        strings = ["a{k}b", "{k}", "a{s}b", "x" * 70000 + "{s}", "{n}", "{m}{m}", "{e}", "", "{s}" * 3000, "{missing}"]
        t = PKG.InsertsTable(table, clock=CLOCK)
        ref = O.Oracle(table, "py", clock=CLOCK)
        for s in strings:
            rst, rout, rvid = ref.interpolate(s)
            got = t.run1(s)
            if rst == "OK_STR":
                assert got == rout, (s[:20], len(got) if isinstance(got, str) else got)
            elif rst == "OK_VALUE":  # a whole-string key: the stored value itself
                assert got == t.value(rvid), s[:20]
            else:
                assert got is PKG.interpolation_engine._NOT_DONE, s[:20]
        for s, (st, payload) in zip(strings, t.run(strings)):
            rst, rout, rvid = ref.interpolate(s)
            assert N.STATUS_NAMES[st] == rst, s[:20]
            assert rst != "OK_STR" or payload == rout, s[:20]
            assert rst != "OK_VALUE" or payload == rvid, s[:20]
        t.close()
    finally:
        x.set_option(N.OPT_VIEWS, 0)


def _window_table(rng):
    """Values of every size class the output windows meet: inline entry texts (<= 28 B), arena
    texts of tens to hundreds of bytes, and multi-KB texts (a tile of those spans many windows or
    goes to the windowed emit kernel)."""
    t = {}
    for j in range(200):
        t["s%d" % j] = "".join(rng.choice("abcdefé€") for _ in range(rng.randint(0, 26)))
        t["m%d" % j] = "".join(rng.choice("mnopq rs") for _ in range(rng.randint(29, 300)))
        t["l%d" % j] = "".join(rng.choice("LMNOP-") for _ in range(rng.randint(900, 5000)))
        t["i%d" % j] = "s%d" % rng.randrange(200)  # {q-{iN}}-style chains: the inner value is a key
        t["q-s%d" % j] = "".join(rng.choice("xyz") for _ in range(rng.randint(1, 40)))
    return t


def _window_strings(rng, n, p_long):
    out = []
    for _ in range(n):
        parts = []
        for _ in range(rng.randint(1, 3)):
            r = rng.random()
            if r < p_long:
                k = "{l%d}" % rng.randrange(200)
            elif r < 0.35:
                k = "{m%d}" % rng.randrange(200)
            elif r < 0.6:
                k = "{q-{i%d}}" % rng.randrange(200)
            else:
                k = "{s%d}" % rng.randrange(200)
            parts.append("".join(rng.choice("ab cd") for _ in range(rng.randint(1, 30))) + k)
        out.append("".join(parts) + "z" * rng.randint(0, 9))
    return out


@pytest.mark.parametrize("p_long", [0.0, 0.004, 0.05])
def test_output_windows_vs_oracle(p_long, fail_commit):
    """Tile outputs from a fraction of the LDS stage to ~40 times it (values of every size class):
    a tile over the stage is deferred to k_emit_windows, which a two-pass views call (the 'defer'
    fixture variants: the LEAN pass, then its deferred subset) launches ONCE for both passes, from
    per-tile records (the subset pass rewrites the first pass's rows of the strings it takes). With
    -DIE_LEAN5=1 the LEAN pass's 13 KB stage and its direct stores past it. Every fixture layout,
    against the oracle."""
    rng = random.Random(int(p_long * 1000) + 5)
    table = _window_table(rng)
    strings = _window_strings(rng, 6000, p_long)
    bad = compare_with_oracle(table, strings)
    assert not bad, [b[:2] for b in bad[:3]]


@pytest.mark.parametrize("reserve", [0, 32])
def test_output_windows_device_views_lean(reserve):
    """The same through ie_interpolate_device_views with the two-pass LEAN path forced and reserved
    output ranges on and off (16-aligned vs unaligned stream-outs), a batch of many tiles, deferred
    tiles in both passes."""
    rng = random.Random(77 + reserve)
    tdict = _window_table(rng)
    strings = _window_strings(rng, 40_000, 0.01)
    x = N.Exec(0)
    x.set_option(N.OPT_VIEWS, 1)
    x.set_option(N.OPT_DEFER, 1)
    x.set_option(N.OPT_RESERVE, reserve)
    table = PKG.InsertsTable(tdict, clock=CLOCK)
    blob, offs = N.pack(strings)
    n = len(strings)
    d_bytes = N.DeviceBuffer.from_numpy(x, np.frombuffer(blob + b"\0" * 16, np.uint8))
    d_off = N.DeviceBuffer.from_numpy(x, np.asarray(offs, np.uint64))
    cap = 64 * len(blob) + (1 << 20)
    r = DevResult(x, n, cap)
    lens = N.DeviceBuffer(x, 4 * n + 4)
    v = N.DevViews(r.bytes.ptr, cap, r.off.ptr, lens.ptr, r.status.ptr, r.vid.ptr, r.total_d.ptr)
    N.check(N.lib().ie_interpolate_device_views(x.h, table.h, None, d_bytes.ptr, d_off.ptr, None, n, ctypes.byref(v)),
            "ie_interpolate_device_views")
    x.sync()
    st = r.status.to_numpy(np.uint8, n)
    starts = r.off.to_numpy(np.uint64, n)
    ln = lens.to_numpy(np.uint32, n).astype(np.uint64)
    ext = int((starts + ln).max())
    out = r.bytes.to_numpy(np.uint8, ext).tobytes()
    assert_views_disjoint(starts, ln, ext)
    ref = O.Oracle(tdict, "py", clock=CLOCK)
    bad = []
    for i, s in enumerate(strings):
        rst, rout, _ = ref.interpolate(s)
        got = out[int(starts[i]):int(starts[i] + ln[i])].decode("utf-8", "surrogatepass") if st[i] == 0 else None
        if N.STATUS_NAMES[st[i]] != rst or (rst == "OK_STR" and got != rout):
            bad.append((i, s[:60], N.STATUS_NAMES[st[i]], rst))
    assert not bad, bad[:3]


def test_deferred_subset_grid_from_a_stale_hint():
    """The deferred subset's grid comes from the exec's previous two-pass call (64 workgroups when
    it deferred nothing) and strides over however many tiles this call defers: a call that defers
    nothing, then one that defers ~100 tiles' worth (keys past 32 bytes leave the LEAN pass), then
    the first again, on one exec, each against the oracle."""
    tdict = dict({"k%d" % i: "v%d" % i for i in range(100)},
                 **{"long_key_number_%030d" % i: "L%d" % i for i in range(50)})
    rng = random.Random(4242)
    light = ["x {k%d} y" % rng.randrange(100) for _ in range(20_000)]
    heavy = [("<{long_key_number_%030d}>" % rng.randrange(50)) if rng.random() < 0.8 else "{k%d}" % rng.randrange(100)
             for _ in range(30_000)]
    x = N.Exec(0)
    x.set_option(N.OPT_VIEWS, 1)
    x.set_option(N.OPT_DEFER, 1)
    table = PKG.InsertsTable(tdict, clock=CLOCK)
    ref = O.Oracle(tdict, "py", clock=CLOCK)
    for k, strings in enumerate([light, heavy, light, heavy]):
        blob, offs = N.pack(strings)
        n = len(strings)
        d_bytes = N.DeviceBuffer.from_numpy(x, np.frombuffer(blob + b"\0" * 16, np.uint8))
        d_off = N.DeviceBuffer.from_numpy(x, np.asarray(offs, np.uint64))
        cap = 4 * len(blob) + (1 << 20)
        r = DevResult(x, n, cap)
        lens = N.DeviceBuffer(x, 4 * n + 4)
        v = N.DevViews(r.bytes.ptr, cap, r.off.ptr, lens.ptr, r.status.ptr, r.vid.ptr, r.total_d.ptr)
        N.check(N.lib().ie_interpolate_device_views(x.h, table.h, None, d_bytes.ptr, d_off.ptr, None, n,
                                                    ctypes.byref(v)), "ie_interpolate_device_views")
        x.sync()  # (the call's telemetry lands: the next call's grid comes from it)
        st = r.status.to_numpy(np.uint8, n)
        starts = r.off.to_numpy(np.uint64, n)
        ln = lens.to_numpy(np.uint32, n).astype(np.uint64)
        ext = int((starts + ln).max())
        out = r.bytes.to_numpy(np.uint8, ext).tobytes()
        assert_views_disjoint(starts, ln, ext)
        bad = []
        for i, s in enumerate(strings):
            rst, rout, _ = ref.interpolate(s)
            got = out[int(starts[i]):int(starts[i] + ln[i])].decode("utf-8", "surrogatepass") if st[i] == 0 else None
            if N.STATUS_NAMES[st[i]] != rst or (rst == "OK_STR" and got != rout):
                bad.append((i, s[:60], N.STATUS_NAMES[st[i]], rst))
        assert not bad, (k, bad[:3])
