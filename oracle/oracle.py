"""TEST INFRASTRUCTURE ONLY — ctypes wrapper around the C oracle (oracle/ie_oracle.c).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module, and
only as the checker / the timed CPU baseline. The product (interpolation-engine_amd/) never does.

The value renderers below restate how the reference turns an insert into splice text:
  py: str(v) with the exact-type rule of interpolation_engine.py:530-531
  rs: value_to_string(v), rust-project/src/interp.rs:314-322 (parity unpinned)
"""
import ctypes
import json
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(HERE, "libie_oracle.so")

DIALECT = {"py": 0, "rs": 1}
KIND_STR, KIND_INT, KIND_LIST, KIND_FLOAT, KIND_BOOL, KIND_NULL, KIND_DICT = range(7)
STATUS_NAMES = ["OK_STR", "OK_VALUE", "E_INTERP", "E_ASSERT_BRACES", "E_ASSERT_TYPE",
                "E_UNHASHABLE", "E_RS_PANIC", "NEEDS_HOST", "DIVERGED", "E_OVERFLOW", "RECURSE"]
VID_NONE, VID_HHMM, VID_HHMMSS = 0xFFFFFFFF, 0xFFFFFFFE, 0xFFFFFFFD


class KV(ctypes.Structure):
    _fields_ = [("key", ctypes.c_char_p), ("key_len", ctypes.c_uint64),
                ("text", ctypes.c_char_p), ("text_len", ctypes.c_uint64),
                ("kind", ctypes.c_int32), ("reserved", ctypes.c_uint32)]


class Clock(ctypes.Structure):
    _fields_ = [("hour", ctypes.c_int32), ("minute", ctypes.c_int32), ("second", ctypes.c_int32)]


class Out(ctypes.Structure):
    _fields_ = [("status", ctypes.c_int32), ("vid", ctypes.c_uint32),
                ("bytes", ctypes.c_void_p), ("len", ctypes.c_uint64)]


def build(force=False):
    """Compile the oracle with gcc (recipe also in oracle/Makefile)."""
    src = os.path.join(HERE, "ie_oracle.c")
    if not force and os.path.exists(SO) and os.path.getmtime(SO) >= os.path.getmtime(src):
        return SO
    subprocess.check_call(["gcc", "-O2", "-fPIC", "-shared", "-pthread", "-o", SO, src])
    return SO


_lib = None


def lib():
    global _lib
    if _lib is None:
        build()
        L = ctypes.CDLL(SO)
        L.ieo_new.restype = ctypes.c_void_p
        L.ieo_new.argtypes = [ctypes.POINTER(KV), ctypes.c_uint64, ctypes.c_int32,
                              ctypes.POINTER(Clock), ctypes.c_int32]
        L.ieo_free.argtypes = [ctypes.c_void_p]
        L.ieo_interpolate.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_uint64, ctypes.POINTER(Out)]
        L.ieo_out_free.argtypes = [ctypes.POINTER(Out)]
        L.ieo_escape.restype = ctypes.c_uint64
        L.ieo_escape.argtypes = [ctypes.c_char_p, ctypes.c_uint64, ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]
        L.ieo_free_bytes.argtypes = [ctypes.c_void_p]
        L.ieo_simple_insertkey.argtypes = [ctypes.c_char_p, ctypes.c_uint64, ctypes.c_int32,
                                           ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)]
        L.ieo_run_batch.restype = ctypes.c_double
        L.ieo_run_batch.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                    ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                    ctypes.c_void_p]
        L.ieo_run_batch_mode.restype = ctypes.c_double
        L.ieo_run_batch_mode.argtypes = L.ieo_run_batch.argtypes + [ctypes.c_int32]
        L.ieo_fnv1a.restype = ctypes.c_uint64
        L.ieo_fnv1a.argtypes = [ctypes.c_void_p, ctypes.c_uint64]
        L.ieo_run_batch_sets.restype = ctypes.c_double
        L.ieo_run_batch_sets.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                         ctypes.c_uint64, ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p,
                                         ctypes.c_void_p, ctypes.c_void_p]
        L.ieo_hash_spans.restype = None
        L.ieo_hash_spans.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                     ctypes.c_uint64, ctypes.c_int32, ctypes.c_void_p]
        _lib = L
    return _lib


def _rs_float(f):
    s = repr(float(f))
    if "e" in s:
        m, e = s.split("e")
        s = "%se%d" % (m, int(e))
    return s


def _rs_vts(v):
    if isinstance(v, str):
        return v
    if isinstance(v, bool):
        return "true" if v else "false"
    if isinstance(v, int):
        return str(v)
    if isinstance(v, float):
        return _rs_float(v)
    if isinstance(v, list):
        return "".join(_rs_vts(x) for x in v)
    return json.dumps(v, separators=(",", ":"), sort_keys=True, ensure_ascii=False)


def render(v, dialect):
    """(kind, splice text) of one insert value."""
    t = type(v)
    kind = {str: KIND_STR, int: KIND_INT, list: KIND_LIST, float: KIND_FLOAT, bool: KIND_BOOL,
            type(None): KIND_NULL, dict: KIND_DICT}.get(t)
    if kind is None:
        raise TypeError("unsupported insert type %r" % t)
    text = str(v) if dialect == "py" else _rs_vts(v)
    return kind, text


def enc(s):
    return s.encode("utf-8", "surrogatepass")


class Oracle:
    def __init__(self, inserts, dialect="py", clock=(12, 34, 56), has_dir=False):
        self.keys = list(inserts.keys())
        self.values = list(inserts.values())
        self._keep = []
        arr = (KV * max(1, len(self.keys)))()
        for i, k in enumerate(self.keys):
            kind, text = render(self.values[i], dialect)
            kb, tb = enc(k), enc(text)
            self._keep += [kb, tb]
            arr[i] = KV(kb, len(kb), tb, len(tb), kind, 0)
        self._arr = arr
        self.clock = Clock(*clock)
        self.h = lib().ieo_new(arr, len(self.keys), DIALECT[dialect], ctypes.byref(self.clock), int(has_dir))

    @classmethod
    def from_kv(cls, kv_ptr, n, dialect="py", clock=(12, 34, 56), has_dir=False):
        o = cls.__new__(cls)
        o.keys = o.values = None
        o._keep = [kv_ptr]
        o.clock = Clock(*clock)
        o.h = lib().ieo_new(ctypes.cast(kv_ptr, ctypes.POINTER(KV)), n, DIALECT[dialect],
                            ctypes.byref(o.clock), int(has_dir))
        return o

    def __del__(self):
        if getattr(self, "h", None):
            lib().ieo_free(self.h)
            self.h = None

    def interpolate(self, s):
        """-> (status name, output str | None, value_id | None)"""
        b = enc(s) if isinstance(s, str) else s
        o = Out()
        lib().ieo_interpolate(self.h, b, len(b), ctypes.byref(o))
        st = STATUS_NAMES[o.status]
        out = None
        if o.status == 0:
            out = ctypes.string_at(o.bytes, o.len).decode("utf-8", "surrogatepass") if o.len else ""
        vid = o.vid if o.status == 1 else None
        lib().ieo_out_free(ctypes.byref(o))
        return st, out, vid

    def run_batch(self, bytes_arr, offsets_arr, n, nthreads=1, status=None, out_len=None, out_hash=None, vid=None,
                  unescape_cmd=False, command_only=False):
        """numpy arrays in/out; returns wall seconds. unescape_cmd: each OK result then goes through
        the `unescape` command (unescape, interpolate again: py:1660-1667), as config 4's step;
        command_only: the `unescape` command alone on each string (item)."""
        def p(a):
            return None if a is None else a.ctypes.data
        mode = 2 if command_only else 1 if unescape_cmd else 0
        return lib().ieo_run_batch_mode(self.h, p(bytes_arr), p(offsets_arr), n, nthreads,
                                        p(status), p(out_len), p(out_hash), p(vid), mode)


def run_batch_sets(oracles, table_id, bytes_arr, offsets_arr, nthreads=1, status=None, out_len=None,
                   out_hash=None, vid=None):
    """A table-set batch: string i against oracles[table_id[i]] (one C call over every string, on
    nthreads threads); returns wall seconds."""
    import numpy as np
    hs = (ctypes.c_void_p * max(1, len(oracles)))(*[o.h for o in oracles])
    tid = np.ascontiguousarray(table_id, dtype=np.uint32)
    def p(a):
        return None if a is None else a.ctypes.data
    return lib().ieo_run_batch_sets(hs, tid.ctypes.data, p(bytes_arr), p(offsets_arr), len(tid), nthreads,
                                    p(status), p(out_len), p(out_hash), p(vid))


def escape(s, unescape=False):
    b = enc(s)
    out = ctypes.c_void_p()
    n = lib().ieo_escape(b, len(b), 1 if unescape else 0, ctypes.byref(out))
    r = ctypes.string_at(out, n).decode("utf-8", "surrogatepass") if n else ""
    lib().ieo_free_bytes(out)
    return r


def simple_insertkey(s, dialect="py"):
    b = enc(s)
    o, l = ctypes.c_uint64(), ctypes.c_uint64()
    r = lib().ieo_simple_insertkey(b, len(b), DIALECT[dialect], ctypes.byref(o), ctypes.byref(l))
    return b[o.value:o.value + l.value].decode("utf-8", "surrogatepass") if r else None


def fnv1a(b):
    return lib().ieo_fnv1a(b, len(b))


def hash_spans(blob, starts, lens, status, nthreads=16):
    """FNV-1a of every OK_STR result of a device batch (0 for status rows): numpy uint8 blob,
    uint64 starts / lengths, uint8 statuses -> uint64 hashes (what run_batch's out_hash holds)."""
    import numpy as np
    blob = np.ascontiguousarray(blob, dtype=np.uint8)
    starts = np.ascontiguousarray(starts, dtype=np.uint64)
    lens = np.ascontiguousarray(lens, dtype=np.uint64)
    status = np.ascontiguousarray(status, dtype=np.uint8)
    n = len(status)
    out = np.zeros(n, np.uint64)
    if n:
        lib().ieo_hash_spans(blob.ctypes.data, starts.ctypes.data, lens.ctypes.data, status.ctypes.data, n,
                             nthreads, out.ctypes.data)
    return out


# ---------------------------------------------------------------------------------------------
# wildcard match / capture: a restatement of the reference's construction (py:553-567) on
# Python's `re` (stdlib: available here and on the GPU box), the checker of k_wildcard
# ---------------------------------------------------------------------------------------------
def wildcard_regex(wildcard_s):
    """py:554 / py:558: '*' -> '〠' -> re.escape -> '(.*)', anchored"""
    import re
    return "^" + re.escape(wildcard_s.replace("*", "〠")).replace("〠", "(.*)") + "$"


def is_wildcard_match(wildcard_s, s):
    """py:553-555 (DOTALL)"""
    import re
    return bool(re.match(wildcard_regex(wildcard_s), s, re.DOTALL))


def get_wildcard_matches(wildcard_s, s):
    """py:557-567: re.findall's groups (a tuple is flattened; a group-less pattern gives the match)"""
    import re
    result = []
    for x in re.findall(wildcard_regex(wildcard_s), s, re.DOTALL):
        if type(x) == tuple:
            result.extend(x)
        else:
            result.append(x)
    return result


def first_wildcard_match(patterns, s):
    """goto_map / replace_map order (py:1704, 1735-1742): the first matching wildcard and its captures"""
    for p, w in enumerate(patterns):
        if is_wildcard_match(w, s):
            return p, get_wildcard_matches(w, s)
    return -1, []


def wildcard_regex_rs(wildcard_s):
    """runtime.rs:1633-1647 / 1754-1775 restated on Python re: '*' -> '(.*)', every other char
    escaped (no U+3020 rule), '$' of the regex crate = Python's \\Z (the end only). Unpinned."""
    import re
    return "^" + "".join("(.*)" if ch == "*" else re.escape(ch) for ch in wildcard_s) + r"\Z"


def first_wildcard_match_rs(patterns, s):
    import re
    for p, w in enumerate(patterns):
        m = re.match(wildcard_regex_rs(w), s, re.DOTALL)
        if m:
            return p, list(m.groups())
    return -1, []
