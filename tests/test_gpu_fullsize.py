"""Whole-batch parity at every BASELINE size: each config's full per-GPU batch goes through the
C ABI on the device, and EVERY string (status, length, FNV-1a of the bytes) is compared with the
oracle (oracle/ie_oracle.c, itself pinned by the reference's golden vectors in
test_oracle_golden.py) running the same inputs on the host's threads. One test per config and
output layout, so a failure names its config.

  config 1  examples/hello_world.json5 through the runner (test_gpu_programs.py)
  config 2  1M strings, single-level {kJ}, 1k inserts                  packed and views output
  config 3  10M strings, nested {q-{iM}}, 100k inserts                 packed and views output
  config 4  12.5M strings (the 100M batch's per-GPU shard): interpolate, then the `unescape`
            command (recursive_unescape + recursive_interpolate, py:1660-1667)
  config 5  10k text_adventure.json5 states, one inserts dict per state in one table set, per
            state every string one loop iteration interpolates (bench.iteration_strings)

Reference: interpolate_inserts, /root/reference/src/interpolation_engine/interpolation_engine.py:
497-541 (restated by the oracle).
"""
import ctypes
import json
import os

import numpy as np
import pytest

import __graft_entry__ as G
from oracle import oracle as O
from tests.conftest import ROOT

pytestmark = pytest.mark.gpu

G.build()
PKG = G.load_package()
N = PKG._native
CLOCK = (12, 34, 56)
THREADS = max(1, min(16, len(os.sched_getaffinity(0))))


def _synth(config):
    h = ctypes.c_void_p()
    N.check(N.lib().ie_synth_create(config, 0, ctypes.byref(h)), "ie_synth_create")
    kvp = ctypes.POINTER(N.KV)()
    nkv = N.lib().ie_synth_kv(h, ctypes.byref(kvp))
    return h, kvp, nkv


def _table(kvp, nkv):
    t = ctypes.c_void_p()
    clk = N.Clock(*CLOCK)
    N.check(N.lib().ie_table_build(ctypes.cast(kvp, ctypes.c_void_p), nkv, 0, ctypes.byref(clk), 0, 0,
                                   ctypes.byref(t)), "ie_table_build")
    return t


def _device_strings(x, h, first, n):
    d_off = N.DeviceBuffer(x, (n + 1) * 8)
    total = ctypes.c_uint64()
    N.check(N.lib().ie_synth_strings_device(x.h, h, first, n, None, 0, d_off.ptr, ctypes.byref(total)), "len")
    d_bytes = N.DeviceBuffer(x, int(total.value) + 16)
    N.check(N.lib().ie_synth_strings_device(x.h, h, first, n, d_bytes.ptr, d_bytes.nbytes, d_off.ptr,
                                            ctypes.byref(total)), "fill")
    return d_off, d_bytes, int(total.value)


class Out:
    """Device outputs of one call in either layout; `starts`/`lens` read them back uniformly."""

    def __init__(self, x, n, cap, views):
        self.n, self.views = n, views
        self.bytes = N.DeviceBuffer(x, cap)
        self.off = N.DeviceBuffer(x, (n + 1) * 8)
        self.len = N.DeviceBuffer(x, 4 * n + 4) if views else None
        self.status = N.DeviceBuffer(x, n + 1)
        self.vid = N.DeviceBuffer(x, 4 * n + 4)
        self.total_d = N.DeviceBuffer(x, 8)
        if views:
            self.desc = N.DevViews(self.bytes.ptr, cap, self.off.ptr, self.len.ptr, self.status.ptr, self.vid.ptr,
                                   self.total_d.ptr)
        else:
            self.desc = N.DevOut(self.bytes.ptr, cap, self.off.ptr, self.status.ptr, self.vid.ptr, self.total_d.ptr)

    def total(self):
        return int(self.total_d.to_numpy(np.uint64, 1)[0])

    def spans(self):
        """(starts, lengths) of every result, uint64"""
        if self.views:
            return self.off.to_numpy(np.uint64, self.n), self.len.to_numpy(np.uint32, self.n).astype(np.uint64)
        oo = self.off.to_numpy(np.uint64, self.n + 1)
        return oo[:-1], np.diff(oo)

    def read(self):
        st = self.status.to_numpy(np.uint8, self.n)
        starts, lens = self.spans()
        # (views: the extent the results reach; reserved ranges leave gaps, *total = sum of lengths)
        ext = int((starts + lens).max()) if self.views and self.n else self.total()
        blob = self.bytes.to_numpy(np.uint8, max(ext, self.total()))
        return st, starts, lens, blob


def interpolate(x, table, d_bytes, d_off, n, cap, views, ids=None):
    o = Out(x, n, cap, views)
    if views:
        N.check(N.lib().ie_interpolate_device_views(x.h, table, ids, d_bytes.ptr, d_off.ptr, None, n,
                                                     ctypes.byref(o.desc)), "ie_interpolate_device_views")
    else:
        N.check(N.lib().ie_interpolate_device_ids(x.h, table, ids, d_bytes.ptr, d_off.ptr, n, ctypes.byref(o.desc)),
                "ie_interpolate_device_ids")
    x.sync()
    assert o.total() <= cap
    return o


def assert_matches_oracle(o, ref_st, ref_len, ref_hash):
    st, starts, lens, blob = o.read()
    bad = np.flatnonzero(st != ref_st)
    assert bad.size == 0, ("status", bad.size, bad[:8], st[bad[:8]], ref_st[bad[:8]])
    ok = st == 0
    bad = np.flatnonzero(ok & (lens != ref_len))
    assert bad.size == 0, ("length", bad.size, bad[:8])
    if o.views:  # a views payload: disjoint results (reserved ranges leave gaps), *total = sum of lengths
        assert int(lens.sum()) == o.total()
        assert_views_disjoint(starts, lens, blob.size)
    else:
        assert int(lens.sum()) == o.total()  # nothing but the results in the payload
    hs = O.hash_spans(blob, starts, lens, st, THREADS)
    bad = np.flatnonzero(hs != ref_hash)
    assert bad.size == 0, ("bytes", bad.size, bad[:8])
    return st, starts, lens


def assert_views_disjoint(starts, lens, total):
    """Every result inside [0, total), no two overlapping (total: the extent the device used)."""
    starts, lens = np.asarray(starts, np.int64), np.asarray(lens, np.int64)
    nz = lens > 0
    s, l = starts[nz], lens[nz]
    assert np.all(s + l <= total) and int(l.sum()) <= total
    o = np.argsort(s, kind="stable")
    assert np.all(s[o][1:] >= (s[o] + l[o])[:-1])


def assert_views_packing(starts, lens, n, tile=256, gaps=False):
    """A views output's 256-string tiles: each tile's strings lie together in input order; without
    reserved ranges the tiles lie together too (no gaps: the extent is the sum of lengths)."""
    starts, lens = starts.astype(np.int64), lens.astype(np.int64)
    if not gaps:
        assert int((starts + lens).max()) == int(lens.sum())
    idx = np.arange(n)
    same_tile = (idx[1:] // tile) == (idx[:-1] // tile)
    follows = starts[1:] == starts[:-1] + lens[:-1]
    assert np.count_nonzero(~follows[same_tile]) == 0


@pytest.mark.parametrize("layout", ["packed", "views", "views-reserve"])
@pytest.mark.parametrize("config,n", [(2, 1_000_000), (3, 10_000_000)], ids=["cfg2-1M", "cfg3-10M"])
def test_full_batch_vs_oracle(config, n, layout):
    """Every string of the BASELINE-size batch against the oracle (status, length, bytes); views-reserve:
    reserved output ranges at 2x the input offsets (IE_OPT_RESERVE 32, the bench's claim)."""
    h, kvp, nkv = _synth(config)
    table = _table(kvp, nkv)
    x = N.Exec(0)
    reserve = layout == "views-reserve"
    if reserve:
        x.set_option(N.OPT_RESERVE, 32)
    d_off, d_bytes, in_total = _device_strings(x, h, 0, n)
    views = layout.startswith("views")
    o = interpolate(x, table, d_bytes, d_off, n, (3 if reserve else 2) * in_total + (1 << 20), views)
    buf = d_bytes.to_numpy(np.uint8, in_total + 1)
    offs = d_off.to_numpy(np.uint64, n + 1)
    ref = O.Oracle.from_kv(ctypes.cast(kvp, ctypes.c_void_p), nkv, "py", clock=CLOCK)
    rst, rlen, rhash = np.zeros(n, np.uint8), np.zeros(n, np.uint64), np.zeros(n, np.uint64)
    ref.run_batch(buf, offs, n, THREADS, rst, rlen, rhash, None)
    st, starts, lens = assert_matches_oracle(o, rst, rlen, rhash)
    assert int(np.count_nonzero(st)) == 0  # the synthetic configs resolve every string
    if views:
        assert_views_packing(starts, lens, n, gaps=reserve)
    N.lib().ie_table_free(table)
    N.lib().ie_synth_free(h)


@pytest.mark.parametrize("layout", ["packed", "views"])
def test_config4_full_step_vs_oracle(layout):
    """Config 4's whole step on its per-GPU batch (12.5M strings, rank 3's shard of the 100M):
    interpolate, then the unescape command on the results; every string against the oracle doing
    the same (ieo_run_batch mode 1). Views: both steps in the views layout, the command fused
    (ie_unescape_cmd_device_views reads the first step's views)."""
    h, kvp, nkv = _synth(4)
    table = _table(kvp, nkv)
    x = N.Exec(0)
    n = 12_500_000
    first = 3 * n
    d_off, d_bytes, in_total = _device_strings(x, h, first, n)
    cap = 2 * in_total + (1 << 20)
    views = layout == "views"
    r = interpolate(x, table, d_bytes, d_off, n, cap, views)
    u = Out(x, n, cap, views)
    if views:
        N.check(N.lib().ie_unescape_cmd_device_views(x.h, table, None, r.bytes.ptr, r.off.ptr, r.len.ptr, n,
                                                     r.status.ptr, ctypes.byref(u.desc)),
                "ie_unescape_cmd_device_views")
    else:
        tmp = Out(x, n, cap, False)
        N.check(N.lib().ie_unescape_cmd_device(x.h, table, None, r.bytes.ptr, r.off.ptr, n, r.status.ptr,
                                               ctypes.byref(tmp.desc), ctypes.byref(u.desc)), "ie_unescape_cmd_device")
    x.sync()
    buf = d_bytes.to_numpy(np.uint8, in_total + 1)
    offs = d_off.to_numpy(np.uint64, n + 1)
    ref = O.Oracle.from_kv(ctypes.cast(kvp, ctypes.c_void_p), nkv, "py", clock=CLOCK)
    rst, rlen, rhash = np.zeros(n, np.uint8), np.zeros(n, np.uint64), np.zeros(n, np.uint64)
    ref.run_batch(buf, offs, n, THREADS, rst, rlen, rhash, None, unescape_cmd=True)
    st, starts, lens = assert_matches_oracle(u, rst, rlen, rhash)
    if views:  # the deferred strings' bytes follow the tiles': gap-free, not in input order
        order = np.argsort(starts[st == 0], kind="stable")
        s_, l_ = starts[st == 0][order].astype(np.int64), lens[st == 0][order].astype(np.int64)
        assert s_[0] == 0 and np.all(s_[1:] == s_[:-1] + l_[:-1])
    names = N.STATUS_NAMES
    assert set(np.unique(st).tolist()) == {names.index("OK_STR"), names.index("E_INTERP")}
    N.lib().ie_table_free(table)
    N.lib().ie_synth_free(h)


def test_config5_10k_states_vs_oracle():
    """Config 5's batch: 10k synthetic text_adventure.json5 states (one inserts dict each, one table
    set), per state every string one loop iteration of its stage interpolates (the benchmark's
    batch); every string against the oracle resolving it with that state's own dict."""
    from interpolation_engine_amd import workloads as Wk
    from bench import iteration_strings  # the benchmark's own batch
    c5 = json.load(open(os.path.join(ROOT, "tests", "golden", "config5_stream.json"), encoding="utf-8"))
    trees = json.load(open(os.path.join(ROOT, "tests", "golden", "config5_trees.json"), encoding="utf-8"))
    stream = {}
    for st in trees["states"]:
        if st["stage"] not in stream:
            stream[st["stage"]] = iteration_strings([t["x"] for t in st["trees"]])
    states = [Wk.state_inserts(c5["defaults"], j) for j in range(10_000)]
    strings, ids = [], []
    for j, ins in enumerate(states):
        strings.extend(stream[ins["stage"]])
        ids.extend([j] * len(stream[ins["stage"]]))
    ids = np.asarray(ids, np.uint32)
    blob, offs = N.pack(strings)
    n = len(strings)
    x = N.Exec(0)
    tset = PKG.InsertsTableSet(states, clock=CLOCK)
    d_bytes = N.DeviceBuffer.from_numpy(x, np.frombuffer(blob + bytes(16), np.uint8))
    d_off = N.DeviceBuffer.from_numpy(x, offs)
    d_ids = N.DeviceBuffer.from_numpy(x, ids)
    buf = np.frombuffer(blob + bytes(1), np.uint8)
    oracles = [O.Oracle(ins, "py", clock=CLOCK) for ins in states]
    rst, rlen, rhash = np.zeros(n, np.uint8), np.zeros(n, np.uint64), np.zeros(n, np.uint64)
    rvid = np.zeros(n, np.uint32)
    O.run_batch_sets(oracles, ids, buf, offs, THREADS, rst, rlen, rhash, rvid)
    for views, defer in ((False, -1), (True, 0), (True, 1)):
        # views: heavy strings in their tiles (IE_OPT_DEFER 0) and in a second pass of their own (1)
        x.set_option(N.OPT_DEFER, defer)
        o = interpolate(x, tset.h, d_bytes, d_off, n, 16 * len(blob) + (1 << 20), views, d_ids.ptr)
        st, _, _ = assert_matches_oracle(o, rst, rlen, rhash)
        # typed whole-string results ({scenario}, {stage}, {history_list}): the same insert; the
        # device's value ids index the set's concatenated dicts, the oracle's one state's dict
        typed = np.flatnonzero(st == N.OK_VALUE)
        assert typed.size >= 3 * 10_000 - 10
        vid = o.vid.to_numpy(np.uint32, n)[typed]
        starts = np.asarray(tset.starts, np.int64)[ids[typed]]
        assert np.array_equal(vid.astype(np.int64) - starts, rvid[typed].astype(np.int64))
    tset.close()
