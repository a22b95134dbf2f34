"""C-ABI boundary checks that need no GPU: the library loads, exports exactly what
include/ie_amd.h declares, refuses to compute without a device (no CPU fallback), and its host
helpers (get_simple_insertkey, the synthetic generator) behave as specified."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

import __graft_entry__ as G
from tests.conftest import ROOT, load_golden

G.build()
PKG = G.load_package()
N = PKG._native


def header_functions():
    src = open(os.path.join(ROOT, "include", "ie_amd.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(ie_[a-z_0-9]+)\s*\(", src)))


def test_header_declares_what_the_binding_uses():
    assert header_functions() == sorted(N.EXPORTS)


def test_library_exports_every_declared_symbol():
    out = subprocess.check_output(["nm", "-D", "--defined-only", N.LIB_PATH], text=True)
    exported = {line.split()[-1] for line in out.splitlines() if " T " in line}
    missing = [f for f in header_functions() if f not in exported]
    assert not missing, missing
    L = N.lib()
    for f in header_functions():
        assert getattr(L, f) is not None


def test_header_constants_match_the_binding():
    """The option and status numbers the Python binding uses are the header's."""
    src = open(os.path.join(ROOT, "include", "ie_amd.h")).read()
    defs = dict(re.findall(r"#define (IE_OPT_[A-Z_]+) (-?\d+)", src))
    assert {k: int(v) for k, v in defs.items()} == {
        "IE_OPT_FAIL_COMMIT": N.OPT_FAIL_COMMIT, "IE_OPT_FAST": N.OPT_FAST,
        "IE_OPT_DEBUG_NOEVAL": N.OPT_DEBUG_NOEVAL, "IE_OPT_TILE": N.OPT_TILE, "IE_OPT_VIEWS": N.OPT_VIEWS,
        "IE_OPT_DEFER": N.OPT_DEFER, "IE_OPT_RESERVE": N.OPT_RESERVE, "IE_OPT_ERROR_KEYS": N.OPT_ERROR_KEYS,
        "IE_OPT_SMALL_ZC": N.OPT_SMALL_ZC}


def test_abi_version():
    assert N.lib().ie_abi_version() == 2


@pytest.mark.skipif(N.lib().ie_device_count() > 0, reason="a GPU is visible")
def test_no_device_means_no_compute():
    """Without a GPU the product refuses to run: it never falls back to a CPU path."""
    h = ctypes.c_void_p()
    assert N.lib().ie_exec_create(0, None, ctypes.byref(h)) == -4  # IE_ERR_NO_DEVICE
    kv = (N.KV * 1)(N.KV(b"a", 1, b"A", 1, 0, 0))
    assert N.lib().ie_table_build(ctypes.cast(kv, ctypes.c_void_p), 1, 0, None, 0, 0, ctypes.byref(h)) == -4
    with pytest.raises(RuntimeError):
        PKG.interpolate_inserts({"a": "A"}, "x{a}")


def test_simple_insertkey_matches_reference_golden():
    for row in load_golden("simple_py.jsonl"):
        got = PKG.get_simple_insertkey(row["s"])
        assert got == row["key"], row


def _synth(config):
    h = ctypes.c_void_p()
    N.check(N.lib().ie_synth_create(config, 0, ctypes.byref(h)), "ie_synth_create")
    return h


@pytest.mark.parametrize("config", [2, 3, 4])
def test_synthetic_strings_follow_the_spec(config):
    h = _synth(config)
    n = 2000 if config < 4 else 20000
    offs = np.zeros(n + 1, np.uint64)
    total = ctypes.c_uint64()
    N.check(N.lib().ie_synth_strings_host(h, 0, n, None, 0, offs.ctypes.data, ctypes.byref(total)), "len")
    buf = np.zeros(int(total.value), np.uint8)
    N.check(N.lib().ie_synth_strings_host(h, 0, n, buf.ctypes.data, buf.size, offs.ctypes.data,
                                          ctypes.byref(total)), "fill")
    lens = np.diff(offs.astype(np.int64))
    assert lens.min() >= 48 and lens.max() <= 80
    assert abs(lens.mean() - 64) < 2
    blob = buf.tobytes()
    kvp = ctypes.POINTER(N.KV)()
    nkv = N.lib().ie_synth_kv(h, ctypes.byref(kvp))
    assert nkv == {2: 1000, 3: 100000, 4: 99999}[config]  # config 4: + "lit", the unescape command's target
    chain = re.compile(r"\{q-(?:\d+|\{i\d+\}|\{a-\{i\d+\}\}|\{a-\{b-\{i\d+\}\}\})\}")
    depth = [0] * 5
    esc = brace_val = missing = 0
    for i in range(n):
        s = blob[int(offs[i]):int(offs[i + 1])].decode("utf-8")
        assert not s.startswith("{")
        assert "〠" not in s
        if config < 4:
            assert "\\" not in s
            refs = re.findall(r"\{k\d+\}" if config == 2 else r"\{q-\{i\d+\}\}", s)
            assert (1 <= len(refs) <= 3) if config == 2 else (1 <= len(refs) <= 2)
            assert s.count("{") == s.count("}") == (1 if config == 2 else 2) * len(refs)
            continue
        # config 4: depth mix 40/30/20/10, 10 % escapes, 2 % brace-bearing values, 1 % misses
        esc += "\\{lit\\}" in s
        rest = s.replace("\\{lit\\}", "")
        brace_val += len(re.findall(r"\{c-\d+\}", rest))
        missing += len(re.findall(r"\{zz-\d+\}", rest))
        rest = re.sub(r"\{(?:c|zz)-\d+\}", "", rest)
        refs = chain.findall(rest)
        for r in refs:
            depth[r.count("{")] += 1
        assert "{" not in chain.sub("", rest) and "}" not in chain.sub("", rest), s
    if config == 4:
        tot = sum(depth)
        for d, share in ((1, 0.40), (2, 0.30), (3, 0.20), (4, 0.10)):
            assert abs(depth[d] / tot - share) < 0.02, depth
        assert abs(esc / n - 0.10) < 0.01 and abs(brace_val / n - 0.02) < 0.005
        assert abs(missing / n - 0.01) < 0.004
    # a window is the same bytes as the full stream
    offs2 = np.zeros(11, np.uint64)
    buf2 = np.zeros(2000, np.uint8)
    N.check(N.lib().ie_synth_strings_host(h, 500, 10, buf2.ctypes.data, buf2.size, offs2.ctypes.data,
                                          ctypes.byref(total)), "window")
    assert buf2[:int(total.value)].tobytes() == blob[int(offs[500]):int(offs[510])]
    N.lib().ie_synth_free(h)


def test_simple_insertkey_fast_paths_match_the_loop():
    # the mirror's pure-Python shortcuts (no '{' first / '}' last; a brace-free '{key}') against the
    # reference's loop (py:484-495) restated here, on random brace strings
    import random

    def loop(content):
        depth = 0
        for i, c in enumerate(content):
            if c == "}":
                depth -= 1
            if (depth == 0) != (i == 0 or i == len(content) - 1):
                return None
            if c == "{":
                depth += 1
        return content[1:-1]
    rng = random.Random(12)
    for _ in range(20000):
        s = "".join(rng.choice("{}ab\\") for _ in range(rng.randrange(0, 9)))
        assert PKG.get_simple_insertkey(s) == loop(s), s
