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


def test_abi_version():
    assert N.lib().ie_abi_version() == 1


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


@pytest.mark.parametrize("config", [2, 3])
def test_synthetic_strings_follow_the_spec(config):
    h = _synth(config)
    n = 2000
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
    assert nkv == (1000 if config == 2 else 100000)
    for i in range(n):
        s = blob[int(offs[i]):int(offs[i + 1])].decode("utf-8")
        assert not s.startswith("{")
        assert "\\" not in s and "〠" not in s
        refs = re.findall(r"\{k\d+\}" if config == 2 else r"\{q-\{i\d+\}\}", s)
        assert (1 <= len(refs) <= 3) if config == 2 else (1 <= len(refs) <= 2)
        assert s.count("{") == s.count("}") == (1 if config == 2 else 2) * len(refs)
    # a window is the same bytes as the full stream
    offs2 = np.zeros(11, np.uint64)
    buf2 = np.zeros(2000, np.uint8)
    N.check(N.lib().ie_synth_strings_host(h, 500, 10, buf2.ctypes.data, buf2.size, offs2.ctypes.data,
                                          ctypes.byref(total)), "window")
    assert buf2[:int(total.value)].tobytes() == blob[int(offs[500]):int(offs[510])]
    N.lib().ie_synth_free(h)
