"""ctypes binding of libie_amd.so (include/ie_amd.h).

The library is the only execution path for the resolver: if it is missing this module raises
at import-use time, and if no HIP device is visible every compute entry point returns
IE_ERR_NO_DEVICE, which is raised as RuntimeError here. There is no CPU fallback.
"""
import ctypes
import os

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("IE_LIB_PATH") or os.path.join(PKG_DIR, "libie_amd.so")  # override: experiments

IE_DIALECT = {"py": 0, "rs": 1}
KIND_STR, KIND_INT, KIND_LIST, KIND_FLOAT, KIND_BOOL, KIND_NULL, KIND_DICT = range(7)
(OK_STR, OK_VALUE, E_INTERP, E_ASSERT_BRACES, E_ASSERT_TYPE, E_UNHASHABLE, E_RS_PANIC, NEEDS_HOST,
 DIVERGED, E_OVERFLOW, RECURSE, E_NO_MATCH, E_NO_NULL) = range(13)
STATUS_NAMES = ["OK_STR", "OK_VALUE", "E_INTERP", "E_ASSERT_BRACES", "E_ASSERT_TYPE",
                "E_UNHASHABLE", "E_RS_PANIC", "NEEDS_HOST", "DIVERGED", "E_OVERFLOW", "RECURSE",
                "E_NO_MATCH", "E_NO_NULL"]
VID_NONE, VID_HHMM, VID_HHMMSS = 0xFFFFFFFF, 0xFFFFFFFE, 0xFFFFFFFD
TABLE_HAS_INSERTS_DIR = 1
TABLE_MUTABLE = 2
OPT_FAIL_COMMIT, OPT_FAST, OPT_DEBUG_NOEVAL, OPT_TILE, OPT_VIEWS, OPT_DEFER, OPT_RESERVE = 1, 2, 3, 4, 5, 7, 8
OPT_ERROR_KEYS = 9
OPT_SMALL_ZC = 10

# every symbol include/ie_amd.h declares (tests check the .so exports exactly these)
EXPORTS = [
    "ie_abi_version", "ie_build_id", "ie_last_error", "ie_device_count",
    "ie_table_build", "ie_table_set_build", "ie_table_set_clock", "ie_table_set_update", "ie_table_set_store", "ie_table_value", "ie_table_free", "ie_table_entries", "ie_table_tables",
    "ie_table_dialect",
    "ie_exec_create", "ie_exec_destroy", "ie_exec_sync", "ie_exec_set_timing", "ie_exec_timing",
    "ie_exec_set_scratch", "ie_exec_set_option", "ie_exec_host_keys",
    "ie_dev_alloc", "ie_dev_free", "ie_copy_h2d", "ie_copy_d2h", "ie_memset_d", "ie_exec_mark",
    "ie_exec_elapsed",
    "ie_interpolate_device", "ie_interpolate_batch", "ie_interpolate", "ie_interpolate_device_ids",
    "ie_interpolate_batch_ids", "ie_interpolate_device_views",
    "ie_unescape_device", "ie_escape_device", "ie_unescape_batch", "ie_escape_batch", "ie_unescape_cmd_device",
    "ie_unescape_cmd_device_views",
    "ie_batch_free", "ie_simple_insertkey",
    "ie_synth_create", "ie_synth_free", "ie_synth_kv", "ie_synth_strings_host",
    "ie_synth_strings_device", "ie_debug_probe",
    "ie_wildcards_build", "ie_wildcards_free", "ie_wildcard_match_device", "ie_wildcard_match_batch",
    "ie_table_replicate", "ie_shard_bounds", "ie_table_arena_stats", "ie_table_set_arena_limit",
    "ie_goto_map", "ie_replace_map", "ie_delete_keys", "ie_map_result_free",
]
WC_MAX_CAP = 16


class KV(ctypes.Structure):
    _fields_ = [("key", ctypes.c_char_p), ("key_len", ctypes.c_uint64),
                ("text", ctypes.c_char_p), ("text_len", ctypes.c_uint64),
                ("kind", ctypes.c_int32), ("reserved", ctypes.c_uint32)]


class Clock(ctypes.Structure):
    _fields_ = [("hour", ctypes.c_int32), ("minute", ctypes.c_int32), ("second", ctypes.c_int32)]


class DevOut(ctypes.Structure):
    _fields_ = [("bytes", ctypes.c_void_p), ("bytes_cap", ctypes.c_uint64),
                ("offsets", ctypes.c_void_p), ("status", ctypes.c_void_p),
                ("value_id", ctypes.c_void_p), ("total", ctypes.c_void_p)]


class DevViews(ctypes.Structure):
    _fields_ = [("bytes", ctypes.c_void_p), ("bytes_cap", ctypes.c_uint64),
                ("offsets", ctypes.c_void_p), ("lengths", ctypes.c_void_p), ("status", ctypes.c_void_p),
                ("value_id", ctypes.c_void_p), ("total", ctypes.c_void_p)]


class BatchRes(ctypes.Structure):
    _fields_ = [("bytes", ctypes.POINTER(ctypes.c_uint8)), ("bytes_len", ctypes.c_uint64),
                ("offsets", ctypes.POINTER(ctypes.c_uint64)), ("status", ctypes.POINTER(ctypes.c_uint8)),
                ("value_id", ctypes.POINTER(ctypes.c_uint32)), ("n", ctypes.c_uint64)]


class MapPair(ctypes.Structure):
    _fields_ = [("key", ctypes.c_char_p), ("key_len", ctypes.c_uint64),
                ("value", ctypes.c_char_p), ("value_len", ctypes.c_uint64)]


class MapResult(ctypes.Structure):
    _fields_ = [("bytes", ctypes.POINTER(ctypes.c_uint8)), ("bytes_len", ctypes.c_uint64),
                ("offsets", ctypes.POINTER(ctypes.c_uint64)), ("status", ctypes.POINTER(ctypes.c_uint8)),
                ("where", ctypes.POINTER(ctypes.c_uint32)), ("chosen", ctypes.POINTER(ctypes.c_int32)),
                ("value_id", ctypes.POINTER(ctypes.c_uint32)), ("n", ctypes.c_uint64)]


def map_result_to_python(res_ptr):
    """Copy an ie_map_result into Python and free it: a list of (bytes, status, where, chosen, value id)."""
    r = res_ptr.contents
    n = r.n
    blob = ctypes.string_at(r.bytes, r.bytes_len) if r.bytes_len else b""

    def arr(p, size, fmt):  # (one copy per array: no ctypes indexing per row)
        return memoryview(ctypes.string_at(p, size * n)).cast(fmt).tolist() if n else []
    o = memoryview(ctypes.string_at(r.offsets, 8 * (n + 1))).cast("Q").tolist()
    st, wh, ch, vid = arr(r.status, 1, "B"), arr(r.where, 4, "I"), arr(r.chosen, 4, "i"), arr(r.value_id, 4, "I")
    out = [(blob[o[i]:o[i + 1]], st[i], wh[i], ch[i], vid[i]) for i in range(n)]
    lib().ie_map_result_free(res_ptr)
    return out


def map_result_columns(res_ptr):
    """Copy an ie_map_result into Python and free it, as columns: (texts as str, statuses, where,
    chosen, value ids). An ASCII result (the common case) is decoded once and sliced."""
    r = res_ptr.contents
    n = r.n
    blob = ctypes.string_at(r.bytes, r.bytes_len) if r.bytes_len else b""
    if n:
        o = memoryview(ctypes.string_at(r.offsets, 8 * (n + 1))).cast("Q").tolist()
        if blob.isascii():
            txt = blob.decode("ascii")
            texts = [txt[a:b] for a, b in zip(o, o[1:])]
        else:
            texts = [dec(blob[a:b]) for a, b in zip(o, o[1:])]

        def arr(p, size, fmt):
            return memoryview(ctypes.string_at(p, size * n)).cast(fmt).tolist()
        cols = (texts, arr(r.status, 1, "B"), arr(r.where, 4, "I"), arr(r.chosen, 4, "i"), arr(r.value_id, 4, "I"))
    else:
        cols = ([], [], [], [], [])
    lib().ie_map_result_free(res_ptr)
    return cols


def map_pairs(pairs):
    """[(key str, value str)] -> (ctypes array of MapPair, the encoded bytes kept alive)"""
    keep = [(enc(k), enc(v)) for k, v in pairs]
    arr = (MapPair * max(1, len(keep)))(*[MapPair(k, len(k), v, len(v)) for k, v in keep])
    return arr, keep


class Timing(ctypes.Structure):
    _fields_ = [("resolve_ms", ctypes.c_float), ("complex_ms", ctypes.c_float),
                ("total_ms", ctypes.c_float), ("n_complex", ctypes.c_uint64), ("n_direct", ctypes.c_uint64),
                ("n_polls", ctypes.c_uint64), ("n_exact", ctypes.c_uint64), ("n_chain_fail", ctypes.c_uint64),
                ("n_deferred", ctypes.c_uint64)]


_lib = None


def signatures():
    """{symbol: (restype, argtypes)} for every entry point of include/ie_amd.h (tests/test_abi.py
    checks this table against the header's prototypes)."""
    vp, u64, i32, u32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int32, ctypes.c_uint32
    pvp = ctypes.POINTER(ctypes.c_void_p)
    return {
        "ie_abi_version": (i32, []),
        "ie_build_id": (ctypes.c_char_p, []),
        "ie_last_error": (ctypes.c_char_p, []),
        "ie_device_count": (i32, []),
        "ie_table_build": (ctypes.c_int, [vp, u64, i32, ctypes.POINTER(Clock), u32, i32, pvp]),
        "ie_table_set_build": (ctypes.c_int, [vp, vp, u32, i32, ctypes.POINTER(Clock), u32, i32, pvp]),
        "ie_table_free": (None, [vp]),
        "ie_table_set_clock": (ctypes.c_int, [vp, ctypes.POINTER(Clock)]),
        "ie_table_set_update": (ctypes.c_int, [vp, vp, vp, vp, u64]),
        "ie_table_set_store": (ctypes.c_int, [vp, vp, vp, u64, vp]),
        "ie_table_value": (ctypes.c_int, [vp, u32, ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_void_p),
                                          ctypes.POINTER(ctypes.c_uint64)]),
        "ie_table_arena_stats": (ctypes.c_int, [vp, ctypes.POINTER(u64), ctypes.POINTER(u64), ctypes.POINTER(u64)]),
        "ie_table_set_arena_limit": (ctypes.c_int, [vp, u64]),
        "ie_goto_map": (ctypes.c_int, [vp, vp, ctypes.c_char_p, u64, vp, u32, ctypes.POINTER(ctypes.POINTER(MapResult))]),
        "ie_replace_map": (ctypes.c_int, [vp, vp, ctypes.c_char_p, u64, vp, vp, vp, u64, vp, u32, i32,
                                          ctypes.POINTER(ctypes.POINTER(MapResult)),
                                          ctypes.POINTER(ctypes.POINTER(MapResult))]),
        "ie_delete_keys": (ctypes.c_int, [vp, vp, vp, u32, vp, vp, u32, i32, ctypes.POINTER(ctypes.POINTER(MapResult))]),
        "ie_map_result_free": (None, [ctypes.POINTER(MapResult)]),
        "ie_table_tables": (u32, [vp]),
        "ie_table_entries": (u64, [vp]),
        "ie_table_dialect": (i32, [vp]),
        "ie_exec_create": (ctypes.c_int, [i32, vp, pvp]),
        "ie_exec_destroy": (None, [vp]),
        "ie_exec_sync": (ctypes.c_int, [vp]),
        "ie_exec_set_timing": (ctypes.c_int, [vp, i32]),
        "ie_exec_timing": (ctypes.c_int, [vp, ctypes.POINTER(Timing)]),
        "ie_exec_set_scratch": (ctypes.c_int, [vp, u64]),
        "ie_exec_set_option": (ctypes.c_int, [vp, i32, ctypes.c_int64]),
        "ie_exec_host_keys": (ctypes.c_int, [vp, vp, u64, ctypes.POINTER(u64)]),
        "ie_dev_alloc": (ctypes.c_int, [i32, u64, pvp]),
        "ie_dev_free": (None, [vp]),
        "ie_copy_h2d": (ctypes.c_int, [vp, vp, vp, u64]),
        "ie_copy_d2h": (ctypes.c_int, [vp, vp, vp, u64]),
        "ie_memset_d": (ctypes.c_int, [vp, vp, i32, u64]),
        "ie_exec_mark": (ctypes.c_int, [vp, u32]),
        "ie_exec_elapsed": (ctypes.c_int, [vp, u32, u32, ctypes.POINTER(ctypes.c_float)]),
        "ie_interpolate_device": (ctypes.c_int, [vp, vp, vp, vp, u64, ctypes.POINTER(DevOut)]),
        "ie_interpolate_batch": (ctypes.c_int, [vp, vp, vp, vp, u64, ctypes.POINTER(ctypes.POINTER(BatchRes))]),
        "ie_interpolate": (ctypes.c_int, [vp, vp, ctypes.c_char_p, u64, ctypes.POINTER(ctypes.POINTER(BatchRes))]),
        "ie_interpolate_device_ids": (ctypes.c_int, [vp, vp, vp, vp, vp, u64, ctypes.POINTER(DevOut)]),
        "ie_interpolate_batch_ids": (ctypes.c_int, [vp, vp, vp, vp, vp, u64, ctypes.POINTER(ctypes.POINTER(BatchRes))]),
        "ie_interpolate_device_views": (ctypes.c_int, [vp, vp, vp, vp, vp, vp, u64, ctypes.POINTER(DevViews)]),
        "ie_unescape_device": (ctypes.c_int, [vp, vp, vp, u64, ctypes.POINTER(DevOut)]),
        "ie_escape_device": (ctypes.c_int, [vp, vp, vp, u64, ctypes.POINTER(DevOut)]),
        "ie_unescape_batch": (ctypes.c_int, [vp, vp, vp, u64, ctypes.POINTER(ctypes.POINTER(BatchRes))]),
        "ie_unescape_cmd_device": (ctypes.c_int, [vp, vp, vp, vp, vp, u64, vp, ctypes.POINTER(DevOut),
                                                  ctypes.POINTER(DevOut)]),
        "ie_escape_batch": (ctypes.c_int, [vp, vp, vp, u64, ctypes.POINTER(ctypes.POINTER(BatchRes))]),
        "ie_unescape_cmd_device_views": (ctypes.c_int, [vp, vp, vp, vp, vp, vp, u64, vp, ctypes.POINTER(DevViews)]),
        "ie_batch_free": (None, [ctypes.POINTER(BatchRes)]),
        "ie_simple_insertkey": (ctypes.c_int, [ctypes.c_char_p, u64, i32, ctypes.POINTER(u64), ctypes.POINTER(u64)]),
        "ie_table_replicate": (ctypes.c_int, [vp, i32, pvp]),
        "ie_debug_probe": (ctypes.c_int, [vp, ctypes.c_char_p, u64, vp]),
        "ie_shard_bounds": (ctypes.c_int, [vp, u64, u32, vp]),
        "ie_wildcards_build": (ctypes.c_int, [vp, vp, u32, i32, i32, pvp]),
        "ie_wildcards_free": (None, [vp]),
        "ie_wildcard_match_device": (ctypes.c_int, [vp, vp, vp, vp, u64, vp, vp, vp, vp]),
        "ie_wildcard_match_batch": (ctypes.c_int, [vp, vp, vp, vp, u64, vp, vp, vp, vp]),
        "ie_synth_create": (ctypes.c_int, [i32, u64, pvp]),
        "ie_synth_free": (None, [vp]),
        "ie_synth_kv": (u64, [vp, ctypes.POINTER(ctypes.POINTER(KV))]),
        "ie_synth_strings_host": (ctypes.c_int, [vp, u64, u64, vp, u64, vp, ctypes.POINTER(u64)]),
        "ie_synth_strings_device": (ctypes.c_int, [vp, vp, u64, u64, vp, u64, vp, ctypes.POINTER(u64)]),
    }


def lib():
    """Load libie_amd.so (raises if it was not built: there is no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError("libie_amd.so is not built (%s); run `python -c \"import __graft_entry__ as g; "
                          "g.build()\"`" % LIB_PATH)
    L = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in signatures().items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    _lib = L
    return L


ERR_CAPACITY = -6  # IE_ERR_CAPACITY


def check(rc, what):
    if rc != 0:
        msg = lib().ie_last_error()
        raise RuntimeError("%s failed (%d): %s" % (what, rc, msg.decode("utf-8", "replace") if msg else ""))


_pack = None


_host_threads = None


def host_threads():
    """Threads for the host-side byte work (IE_HOST_THREADS, else the cores, at most 8; read once)."""
    global _host_threads
    if _host_threads is None:
        v = int(os.environ.get("IE_HOST_THREADS", "0") or 0)
        _host_threads = v if v > 0 else max(1, min(8, os.cpu_count() or 1))
    return _host_threads


def pack_module():
    """The store packer (csrc/ie_pack.c, built in-tree by __graft_entry__.build next to the library)."""
    global _pack
    if _pack is None:
        try:
            from . import _ie_pack
        except ImportError as e:
            raise RuntimeError("the store packer _ie_pack is not built (run __graft_entry__.build()): %s" % e)
        _pack = _ie_pack
    return _pack


def enc(s):
    return s.encode("utf-8", "surrogatepass")


def dec(b):
    return b.decode("utf-8", "surrogatepass")


class Exec:
    """An ie_exec: device, HIP stream, workspace. `stream` is a raw hipStream_t (int) or None."""

    def __init__(self, device=0, stream=None):
        h = ctypes.c_void_p()
        check(lib().ie_exec_create(device, stream, ctypes.byref(h)), "ie_exec_create")
        self.h = h
        self.device = device

    def host_keys(self):
        """{string index: [key, ...]}: the keys the last interpolation call could not look up on
        the device (IE_NEEDS_HOST), ie_exec_host_keys."""
        used = ctypes.c_uint64()
        check(lib().ie_exec_host_keys(self.h, None, 0, ctypes.byref(used)), "ie_exec_host_keys")
        if not used.value:
            return {}
        buf = ctypes.create_string_buffer(used.value)
        check(lib().ie_exec_host_keys(self.h, buf, used.value, ctypes.byref(used)), "ie_exec_host_keys")
        raw, out, k = buf.raw, {}, 0
        while k + 8 <= len(raw):
            idx = int.from_bytes(raw[k:k + 4], "little")
            n = int.from_bytes(raw[k + 4:k + 8], "little")
            out.setdefault(idx, []).append(dec(raw[k + 8:k + 8 + n]))
            k += 8 + ((n + 3) & ~3)
        return out

    def close(self):
        if getattr(self, "h", None):
            lib().ie_exec_destroy(self.h)
            self.h = None

    __del__ = close

    def sync(self):
        check(lib().ie_exec_sync(self.h), "ie_exec_sync")

    def set_timing(self, on):
        check(lib().ie_exec_set_timing(self.h, 1 if on else 0), "ie_exec_set_timing")

    def set_option(self, option, value):
        check(lib().ie_exec_set_option(self.h, option, value), "ie_exec_set_option")

    def timing(self):
        t = Timing()
        check(lib().ie_exec_timing(self.h, ctypes.byref(t)), "ie_exec_timing")
        return t

    def mark(self, slot):
        check(lib().ie_exec_mark(self.h, slot), "ie_exec_mark")

    def elapsed(self, a, b):
        ms = ctypes.c_float()
        check(lib().ie_exec_elapsed(self.h, a, b, ctypes.byref(ms)), "ie_exec_elapsed")
        return ms.value


class DeviceBuffer:
    """A device allocation owned by libie_amd (hipMalloc), with numpy copies in and out."""

    def __init__(self, x, nbytes, device=None):
        self.x = x
        self.nbytes = int(nbytes)
        p = ctypes.c_void_p()
        check(lib().ie_dev_alloc(x.device if device is None else device, max(self.nbytes, 16), ctypes.byref(p)),
              "ie_dev_alloc")
        self.p = p

    @property
    def ptr(self):
        return self.p.value

    @classmethod
    def from_numpy(cls, x, arr):
        import numpy as np
        arr = np.ascontiguousarray(arr)
        b = cls(x, arr.nbytes)
        check(lib().ie_copy_h2d(x.h, b.p, arr.ctypes.data, arr.nbytes), "ie_copy_h2d")
        return b

    def to_numpy(self, dtype, count, offset_bytes=0):
        import numpy as np
        out = np.empty(count, dtype=dtype)
        if out.nbytes:
            check(lib().ie_copy_d2h(self.x.h, out.ctypes.data, self.ptr + offset_bytes, out.nbytes), "ie_copy_d2h")
        return out

    def zero(self):
        check(lib().ie_memset_d(self.x.h, self.p, 0, self.nbytes), "ie_memset_d")

    def free(self):
        if getattr(self, "p", None) and self.p.value:
            lib().ie_dev_free(self.p)
            self.p = ctypes.c_void_p()

    __del__ = free


def batch_to_python(res_ptr):
    """Copy an ie_batch into Python: (list[bytes], list[int status], list[int vid])."""
    r = res_ptr.contents
    n = r.n
    if n <= 16:  # (a scalar call: no numpy views, a few ctypes reads)
        o = [r.offsets[i] for i in range(n + 1)] if n else [0]
        blob = ctypes.string_at(r.bytes, r.bytes_len) if r.bytes_len else b""
        st = [r.status[i] for i in range(n)]
        vid = [r.value_id[i] for i in range(n)]
        lib().ie_batch_free(res_ptr)
        return [blob[o[i]:o[i + 1]] for i in range(n)], st, vid
    import numpy as np
    offs = np.ctypeslib.as_array(r.offsets, shape=(n + 1,)).copy() if n else np.zeros(1, np.uint64)
    st = np.ctypeslib.as_array(r.status, shape=(n,)).copy() if n else np.zeros(0, np.uint8)
    vid = np.ctypeslib.as_array(r.value_id, shape=(n,)).copy() if n else np.zeros(0, np.uint32)
    blob = ctypes.string_at(r.bytes, r.bytes_len) if r.bytes_len else b""
    lib().ie_batch_free(res_ptr)
    o = offs.tolist()
    outs = [blob[o[i]:o[i + 1]] for i in range(n)]
    return outs, st.tolist(), vid.tolist()


_PY_PACK = os.environ.get("IE_PY_PACK") == "1"  # (A/B: the Python packing)


def pack(strings):
    """list[str|bytes] -> (bytes blob, uint64 offsets array); in C (_ie_pack.pack_strs) when the
    packer is built"""
    import numpy as np
    if not _PY_PACK:
        try:
            blob, o = pack_module().pack_strs(strings)
            return blob, np.frombuffer(o, dtype=np.uint64).copy()
        except (RuntimeError, TypeError):  # (the packer not built, or items other than str / bytes)
            pass
    memo = {}  # batches repeat strings (a task's texts once per state): each encoded once

    def one(s):
        if type(s) is str:
            b = memo.get(s)
            if b is None:
                b = memo[s] = enc(s)
            return b
        return bytes(s)
    bs = [one(s) for s in strings]
    offs = np.zeros(len(bs) + 1, dtype=np.uint64)
    if bs:
        offs[1:] = np.cumsum([len(b) for b in bs], dtype=np.uint64)
    return b"".join(bs), offs
