"""Drop-in mirror of the reference's interpolation surface, resolved by the HIP kernels.

Same names, argument meaning and error behaviour as src/interpolation_engine/interpolation_engine.py:
  InterpolationException           py:426-428
  get_interpdata(inserts, key)     py:430-467
  get_simple_insertkey(content)    py:477-495
  interpolate_inserts(inserts, s)  py:497-541   -> one string through libie_amd (a batch of one)
  recursive_unescape / _escape     py:1436-1460 -> every string leaf in ONE device batch
  recursive_interpolate(inserts,x) py:1462-1494 -> every string leaf in ONE device batch
plus the batch entry the GPU is for:
  interpolate_batch(inserts, strings) -> list of results (str / typed value / exception instance)

Errors map from the per-string device status: E_INTERP -> InterpolationException,
E_ASSERT_* -> AssertionError, E_UNHASHABLE -> TypeError (py:450 `in` on an unhashable key).
The reference loops forever on self-referential inserts; here such strings stop at the
IE_ITER_CAP / IE_SIZE_CAP caps (include/ie_amd.h) and raise RecursionError.

`get_interpdata` and `get_simple_insertkey` are the two scalar helpers the reference's callers
use for control flow (recursive_interpolate's for/serial branch, validate_program); they are
host glue with the reference's exact semantics. Every string interpolation, escape and
unescape runs on the device; without libie_amd.so or a GPU the calls raise.
"""
import copy
import contextlib
import ctypes
import datetime as _dt
import gc
import json
import os
import re
import time

from . import _native as N

insert_start = "{"
insert_stop = "}"
escape = "\\"
inserts_dir = None  # py:44 — when set, get_interpdata falls back to its files (py:452-461)


DELETE = object()  # InsertsTableSet.update: remove the key (`del inserts[key]`)
_NOT_DONE = object()  # InsertsTableSet.run1: the string needs results() (a failure, an inserts-directory key)
_IN_TABLE = object()  # InsertsTableSet.values: a str / int the table's mirror holds (value() reads it)


@contextlib.contextmanager
def _gc_paused():
    """The cyclic collector off for a bulk step (a store, a build, a map run): the callers' heaps hold
    millions of objects, and a full collection in the middle costs tens of ms; the steps create no
    cycles of their own."""
    was = gc.isenabled()
    gc.disable()
    try:
        yield
    finally:
        if was:
            gc.enable()


class InterpolationException(Exception):
    # Caught in goto_map to trigger the 'NULL' key (py:426-428).
    pass


# ------------------------------------------------------------------------------------------
# value rendering (the splice text of py:531 / interp.rs:71-80, value_to_string interp.rs:314)
# ------------------------------------------------------------------------------------------
_KIND = {str: N.KIND_STR, int: N.KIND_INT, list: N.KIND_LIST, float: N.KIND_FLOAT,
         bool: N.KIND_BOOL, type(None): N.KIND_NULL, dict: N.KIND_DICT}


def _rs_float(f):
    s = repr(float(f))
    if "e" in s:
        m, e = s.split("e")
        s = "%se%d" % (m, int(e))
    return s


def _rs_value_to_string(v):
    if isinstance(v, str):
        return v
    if isinstance(v, bool):
        return "true" if v else "false"
    if isinstance(v, int):
        return str(v)
    if isinstance(v, float):
        return _rs_float(v)
    if isinstance(v, list):
        return "".join(_rs_value_to_string(x) for x in v)
    return json.dumps(v, separators=(",", ":"), sort_keys=True, ensure_ascii=False)


def render(v, dialect="py"):
    kind = _KIND.get(type(v))
    if kind is None:
        raise TypeError("insert values must be JSON types, got %r" % type(v))
    return kind, (str(v) if dialect == "py" else _rs_value_to_string(v))


# ------------------------------------------------------------------------------------------
# device context
# ------------------------------------------------------------------------------------------
_execs = {}


def get_exec(device=0):
    x = _execs.get(device)
    if x is None:
        x = _execs[device] = N.Exec(device)
        # the missing key of every failed lookup comes back with its string (the message names it)
        x.set_option(N.OPT_ERROR_KEYS, 1)
    return x


class InsertsTableSet:
    """Immutable device snapshots of several inserts dicts in ONE device table (a table set,
    include/ie_amd.h ie_table_set_build): every string names the dict it resolves against.
    This is the batch form of get_interpdata for many forked interpreter states (config 5)."""

    def __init__(self, dicts, dialect="py", clock=None, device=0, has_inserts_dir=False, mutable=False):
        self.clock_pinned = clock is not None  # else the wall clock at build (set_clock re-reads it)
        if clock is None:
            now = _dt.datetime.now()
            clock = (now.hour, now.minute, now.second)
        self.clock = tuple(clock)
        self.dialect = dialect
        self.device = device
        self.has_dir = bool(has_inserts_dir)
        self.dicts = list(dicts)
        self.keys, self.values, starts = [], [], [0]
        for d in self.dicts:
            self.keys.extend(d.keys())
            self.values.extend(d.values())
            starts.append(len(self.keys))
        self.starts = starts
        # the ie_kv records of every dict in one native pass (csrc/ie_pack.c: pointers into the
        # str objects, the texts that are not ASCII transcoded across host threads): a table set of
        # many states holds ~10^5 entries
        with _gc_paused():
            kvb, stb, keep = N.pack_module().pack_dicts([d if isinstance(d, dict) else dict(d) for d in self.dicts],
                                                         render, dialect, N.host_threads())
        cb = ctypes.c_char * len(kvb)
        h = ctypes.c_void_p()
        clk = N.Clock(*self.clock)
        st = (ctypes.c_char * len(stb)).from_buffer(stb)
        N.check(N.lib().ie_table_set_build(cb.from_buffer(kvb), st, len(self.dicts),
                                           N.IE_DIALECT[dialect], ctypes.byref(clk),
                                           (N.TABLE_HAS_INSERTS_DIR if has_inserts_dir else 0) |
                                           (N.TABLE_MUTABLE if mutable else 0), device,
                                           ctypes.byref(h)), "ie_table_set_build")
        del keep  # (the records pointed into these until the build returned)
        self.h = h

    def close(self):
        if getattr(self, "h", None):
            N.lib().ie_table_free(self.h)
            self.h = None

    __del__ = close

    def set_clock(self, clock):
        """Re-read the clock without a rebuild; False when the table must be rebuilt instead."""
        clk = N.Clock(*clock)
        if N.lib().ie_table_set_clock(self.h, ctypes.byref(clk)) != 0:
            return False
        self.clock = tuple(clock)
        return True

    def value(self, vid):
        if vid == N.VID_HHMM:
            return "%02d:%02d" % self.clock[:2]
        if vid == N.VID_HHMMSS:
            return "%02d:%02d:%02d" % self.clock
        v = self.values[vid]
        if v is _IN_TABLE:  # a str / int stored by update(): read back from the table's mirror
            if not getattr(self, "h", None):
                raise RuntimeError("the table set is closed: a stored value is read back from its table")
            k, p, n = ctypes.c_int32(), ctypes.c_void_p(), ctypes.c_uint64()
            N.check(N.lib().ie_table_value(self.h, vid, ctypes.byref(k), ctypes.byref(p), ctypes.byref(n)),
                    "ie_table_value")
            text = N.dec(ctypes.string_at(p.value, n.value)) if n.value else ""
            return int(text) if k.value == N.KIND_INT else text
        return v

    def table_keys(self, t):
        return list(self.dicts[t].keys())  # the live dict (as py:467's message reads it)

    def update(self, changes):
        """set_interpdata on the device copy (py:470-471 `inserts[key] = value`, or DELETE for
        `del`), without a rebuild (ie_table_set_store): changes = [(dict index, key, value)].
        The caller's dicts are not touched (the states the table set was built from are usually the
        caller's own, already updated). False when the library found no placement for a new key:
        then rebuild the table set. The packing is native (csrc/ie_pack.c: ie_kv records over the
        str objects' own UTF-8) and the library hands out the value ids (a rewrite keeps its key's,
        a delete frees it); the stored values land in self.values under those ids."""
        n = len(changes)
        if n == 0:
            return True
        P = N.pack_module()
        tp = time.perf_counter()
        if n < 4096:  # (a few stores: no collection to fear, and the pause costs a µs of its own)
            return self._store(P, changes, n, tp)
        with _gc_paused():  # (no cyclic collection over the caller's heap in the middle of a store)
            return self._store(P, changes, n, tp)

    def _store(self, P, changes, n, tp):
        kv, tids, keep = P.pack(changes, len(self.dicts), DELETE, render, self.dialect, N.host_threads())
        vids = bytearray(4 * n)
        cv = ctypes.c_char * (4 * n)
        t0 = time.perf_counter()
        rc = N.lib().ie_table_set_store(self.h, (ctypes.c_char * len(kv)).from_buffer(kv), cv.from_buffer(tids), n,
                                        cv.from_buffer(vids))
        t1 = time.perf_counter()
        del keep  # (the records point into these texts until the call returns)
        if rc == N.ERR_CAPACITY:
            return False
        N.check(rc, "ie_table_set_store")
        P.assign(self.values, changes, vids, DELETE, _IN_TABLE)
        # (where a store call's time goes: packing, the library, the value list)
        self.last_update_native_s = t1 - t0
        self.last_update_split_s = (t0 - tp, t1 - t0, time.perf_counter() - t1)
        return True

    def set_arena_limit(self, nbytes):
        """Lower the text arena's limit (update then reports False, a rebuild, once it is reached)."""
        N.check(N.lib().ie_table_set_arena_limit(self.h, nbytes), "ie_table_set_arena_limit")

    def arena_stats(self):
        """(bytes in use, live bytes, compactions) of the table set's text arena."""
        b, l, c = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
        N.check(N.lib().ie_table_arena_stats(self.h, ctypes.byref(b), ctypes.byref(l), ctypes.byref(c)),
                "ie_table_arena_stats")
        return b.value, l.value, c.value

    # --------------------------------------------------------------------------------------
    def run(self, strings, table_ids=None, exec_=None):
        """Resolve a list of str on the device -> list of (status, payload); string i against dict
        table_ids[i] (all against dict 0 when table_ids is None); exec_: the caller's ie_exec
        (one per host thread), else this device's shared one."""
        x = exec_ or get_exec(self.device)
        res = ctypes.POINTER(N.BatchRes)()
        if table_ids is None and len(strings) == 1 and type(strings[0]) is str:
            # a scalar call (interpolate_inserts): the string's bytes and two offsets, no numpy
            b = N.enc(strings[0])
            offs1 = (ctypes.c_uint64 * 2)(0, len(b))
            N.check(N.lib().ie_interpolate_batch(x.h, self.h, b, offs1, 1, ctypes.byref(res)), "ie_interpolate_batch")
            outs, sts, vids = N.batch_to_python(res)
            return [(sts[0], N.dec(outs[0]) if sts[0] == N.OK_STR else (vids[0] if sts[0] == N.OK_VALUE else None))]
        blob, offs = N.pack(strings)
        bp = ctypes.c_char_p(blob)
        if table_ids is None:
            N.check(N.lib().ie_interpolate_batch(x.h, self.h, ctypes.cast(bp, ctypes.c_void_p),
                                                 offs.ctypes.data, len(strings), ctypes.byref(res)),
                    "ie_interpolate_batch")
        else:
            import numpy as np
            ids = np.ascontiguousarray(table_ids, dtype=np.uint32)
            if ids.size != len(strings):
                raise ValueError("one table id per string")
            N.check(N.lib().ie_interpolate_batch_ids(x.h, self.h, ids.ctypes.data, ctypes.cast(bp, ctypes.c_void_p),
                                                     offs.ctypes.data, len(strings), ctypes.byref(res)),
                    "ie_interpolate_batch_ids")
        outs, sts, vids = N.batch_to_python(res)
        memo = {}  # (many states give the same text: each distinct output decoded once)

        def text(o):
            t = memo.get(o)
            if t is None:
                t = memo[o] = N.dec(o)
            return t
        return [(st, text(o) if st == N.OK_STR else (vids[i] if st == N.OK_VALUE else None))
                for i, (o, st) in enumerate(zip(outs, sts))]

    def run1(self, s):
        """One str against dict 0 (a scalar interpolate_inserts): its result when the device
        resolved it (a text or a stored value), else _NOT_DONE (the caller takes results(), which
        builds the failure or completes an inserts-directory key). The same library call as run(),
        without the list plumbing."""
        x = get_exec(self.device)
        b = N.enc(s)
        res = ctypes.POINTER(N.BatchRes)()
        lib = N.lib()
        N.check(lib.ie_interpolate_batch(x.h, self.h, b, (ctypes.c_uint64 * 2)(0, len(b)), 1, ctypes.byref(res)),
                "ie_interpolate_batch")
        r = res.contents
        st, vid, o0, o1 = r.status[0], r.value_id[0], r.offsets[0], r.offsets[1]
        out = ctypes.string_at(r.bytes, o1)[o0:] if st == N.OK_STR and o1 else b""
        lib.ie_batch_free(res)
        if st == N.OK_STR:
            return N.dec(out)
        if st == N.OK_VALUE:
            return self.value(vid)
        return _NOT_DONE

    def results(self, strings, table_ids=None):
        """Like interpolate_inserts on each string; failures come back as exception instances."""
        ids = [0] * len(strings) if table_ids is None else (
            table_ids.tolist() if hasattr(table_ids, "tolist") else list(table_ids))
        out = []
        got = self.run(strings, table_ids)
        # the keys the device could not look up (IE_NEEDS_HOST), also those built from values, and
        # the missing keys of the failed lookups (IE_E_INTERP, IE_OPT_ERROR_KEYS)
        need = any(st == N.E_INTERP or (self.has_dir and st == N.NEEDS_HOST) for st, _ in got)
        host_keys = get_exec(self.device).host_keys() if need else {}
        for i, (s, t, (st, payload)) in enumerate(zip(strings, ids, got)):
            if st == N.OK_STR:
                out.append(payload)
            elif st == N.OK_VALUE:
                out.append(self.value(payload))
            elif self.has_dir and inserts_dir and (st == N.NEEDS_HOST or (st == N.E_INTERP and _dir_bad)):
                out.append(self._host_complete(s, t, st, host_keys.get(i, [])))
            else:
                out.append(_exception(s, st, self.table_keys(t), host_keys.get(i), self.has_dir))
        return out

    def _host_complete(self, s, t, st, device_keys=()):
        """The inserts-directory lookups the device hands to the host (get_interpdata's file
        fallback, py:452-461). IE_NEEDS_HOST: a key that is not a canonical relative file name
        (os.path.join may leave the directory, so no snapshot holds it): the host opens the files
        the string's literal keys name (and keys inside what it read), adds what it finds to the
        string's dict and resolves the string on the device again; a key whose files are missing is
        the reference's miss. IE_E_INTERP with unreadable files in the directory: the reference
        raises that file's error when its key is looked up. Returns a result or an exception."""
        keys = _literal_keys(s)
        base = self.dicts[t]
        if st == N.E_INTERP:
            # the reference looks keys up innermost-rightmost first (py:520, rfind): the first
            # literal key, in that order, that neither the dict nor the snapshot holds is the
            # lookup that failed; a file the snapshot could not read raises its own error there
            snap = _dir_snap.get(inserts_dir)
            have = snap[2] if snap else {}
            for k in reversed(keys):
                if k in base or k in have:
                    continue
                e = _dir_bad.get(os.path.join(inserts_dir, k))
                return e if e is not None else _exception(s, st, self.table_keys(t), device_keys, True)
            return _exception(s, st, self.table_keys(t), device_keys, True)
        extras, missing = {}, set()
        for _ in range(8):
            found = list(device_keys) + keys + [k for v in extras.values() if isinstance(v, str) for k in _literal_keys(v)]
            cands = [k for k in dict.fromkeys(found)
                     if not _canonical_key(k) and k not in base and k not in extras and k not in missing]
            if not cands:
                break
            for k in cands:
                try:
                    extras[k] = _read_dir_key(k)
                except FileNotFoundError:
                    missing.add(k)
                except Exception as e:  # noqa: BLE001 — IsADirectoryError, UnicodeDecodeError, a JSON5 error
                    return e
            tbl = InsertsTable(base, dialect=self.dialect, clock=self.clock, device=self.device,
                               has_inserts_dir=True, extra=extras)
            try:
                st2, payload = tbl.run([s])[0]
                if st2 == N.OK_STR:
                    return payload
                if st2 == N.OK_VALUE:
                    return tbl.value(payload)
                if st2 != N.NEEDS_HOST:
                    return _exception(s, st2, tbl.table_keys(0))
                # the next key the device could not look up (built from what was just added too)
                device_keys = list(device_keys) + get_exec(self.device).host_keys().get(0, [])
            finally:
                tbl.close()
        for k in sorted(missing):
            try:
                get_interpdata(base, k)
            except InterpolationException as e:
                return e
        return _exception(s, N.NEEDS_HOST, self.table_keys(t))


class InsertsTable(InsertsTableSet):
    """An immutable device snapshot of one inserts dict (get_interpdata's view of it)."""

    dir_key = None

    def __init__(self, inserts, dialect="py", clock=None, device=0, has_inserts_dir=False, extra=None):
        merged = inserts if not extra else {**extra, **inserts}  # the inserts win (py:450 before 452)
        super().__init__([merged], dialect=dialect, clock=clock, device=device, has_inserts_dir=has_inserts_dir,
                         mutable=True)
        self._snapshot = (dict(inserts), {k: render(v, dialect)[1] for k, v in inserts.items()
                                          if isinstance(v, (list, dict))})
        self._version = getattr(inserts, "version", None)

    def refresh(self, inserts):
        """Bring this snapshot up to date with `inserts` in place (ie_table_set_update) when only a
        few keys changed: False when a rebuild is the better (or the only) way."""
        if self.dicts[0] is not inserts:  # (a merged inserts-directory snapshot, or another dict)
            return False
        snap, mutable = self._snapshot
        logged = inserts.keys_since(self._version) if isinstance(inserts, VersionedInserts) else None
        if logged is not None:  # only the keys stored since this snapshot (VersionedInserts' log)
            changes = [(0, k, inserts[k] if k in inserts else DELETE) for k in logged
                       if (k in inserts and (k not in snap or snap[k] is not inserts[k]
                                             or isinstance(inserts[k], (list, dict)))) or (k not in inserts and k in snap)]
            if not self.update(changes):
                return False
            for _, k, v in changes:
                if v is DELETE:
                    snap.pop(k, None)
                    mutable.pop(k, None)
                    continue
                snap[k] = v
                if isinstance(v, (list, dict)):
                    mutable[k] = render(v, self.dialect)[1]
                else:
                    mutable.pop(k, None)
            self._version = inserts.version
            return True
        changes = [(0, k, v) for k, v in inserts.items()
                   if k not in snap or snap[k] is not v
                   or (k in mutable and render(v, self.dialect)[1] != mutable[k])]
        changes += [(0, k, DELETE) for k in snap if k not in inserts]
        if len(changes) > max(64, len(inserts) // 4) or not self.update(changes):
            return False
        self._snapshot = (dict(inserts), {k: render(v, self.dialect)[1] for k, v in inserts.items()
                                          if isinstance(v, (list, dict))})
        self._version = getattr(inserts, "version", None)
        return True

    def matches(self, inserts):
        """Is this still a snapshot of `inserts`? O(1) for a VersionedInserts, else O(len)."""
        v = getattr(inserts, "version", None)
        if v is not None:
            return v == self._version
        snap, mutable = self._snapshot
        if len(inserts) != len(snap):
            return False
        for k, v in inserts.items():
            if k not in snap or snap[k] is not v:
                return False
        for k, text in mutable.items():  # lists/dicts may have been mutated in place
            if render(inserts[k], self.dialect)[1] != text:
                return False
        return True


def _exception(s, st, keys, missing=None, has_dir=False):
    """The exception the reference raises for a string the device reported as `st`; `missing`: the
    keys the device recorded for it (IE_OPT_ERROR_KEYS), the last one is the failed lookup."""
    if st == N.E_INTERP:
        if missing:
            return _missing_key_exception(missing[-1], keys, has_dir)
        return InterpolationException(
            "Could not resolve an interpolation in %r. Available interpolation data keys are %r." % (s, keys))
    if st == N.E_ASSERT_BRACES:
        return AssertionError("Error: The following content has an uneven number of '{' and '}':\n\n\"\"\"%s\n\"\"\"" % s)
    if st == N.E_ASSERT_TYPE:
        return AssertionError("Error: trying to interpolate a variable of a type other than str, int or list into %r." % s)
    if st == N.E_UNHASHABLE:
        return TypeError("unhashable type used as an interpolation key in %r" % s)
    if st == N.E_RS_PANIC:
        return RuntimeError("rust dialect: unwrap() on a '}{' leftover in %r" % s)
    if st == N.DIVERGED:
        return RecursionError("interpolation of %r does not terminate (self-referential inserts)" % s)
    if st == N.NEEDS_HOST:
        return NotImplementedError("a key of %r names a path outside the inserts directory's snapshot "
                                   "('/', '.', '..' or NUL in the key): not resolved on the device path" % s)
    return RuntimeError("device status %s for %r" % (N.STATUS_NAMES[st] if st < len(N.STATUS_NAMES) else st, s))


def _missing_key_exception(key, keys, has_dir):
    """get_interpdata's messages for a key it does not find (py:430-467): an ARGn key, the empty
    key, or any other (with the inserts directory it also looked in)."""
    if _is_arg_key(key):
        return InterpolationException("Argument interpolation key '%s' is used, but the user passed less than %s "
                                      "program arguments." % (key, key[3:]))
    if key == "":
        return InterpolationException("Tried to interpolate empty string ''.")
    detail = " in interpdata" + (" or inserts directory '%s'" % inserts_dir if has_dir and inserts_dir else "")
    return InterpolationException("Could not find variable '%s'%s. Available interpolation data keys are %r."
                                  % (key, detail, list(keys)))


class VersionedInserts(dict):
    """A dict that counts its mutations, so table_for() recognises an unchanged inserts dict in
    O(1) instead of comparing every value (use it as the runner's `state['inserts']`). Mutating a
    list or dict value in place is not a mutation of this dict: bump() after doing that.
    `d[k] = v` and `del d[k]` are also logged (version, key), so a table refreshes from the keys
    stored since its version instead of comparing the whole dict; the log covers the versions after
    log_base (other mutators, bump() and a full log start it again)."""
    __slots__ = ("version", "log", "log_base")
    _LOG_MAX = 64

    def __init__(self, *a, **k):
        super().__init__(*a, **k)
        self.version = 0
        self.log = []
        self.log_base = 0

    def bump(self):
        self.version += 1
        self.log, self.log_base = [], self.version

    def __setitem__(self, k, v):
        self.version += 1
        dict.__setitem__(self, k, v)
        self._logged(k)

    def __delitem__(self, k):
        self.version += 1
        dict.__delitem__(self, k)
        self._logged(k)

    def _logged(self, k):
        if len(self.log) >= self._LOG_MAX:
            self.log, self.log_base = [], self.version
        else:
            self.log.append((self.version, k))

    def keys_since(self, version):
        """The keys stored or deleted after `version`, or None when the log does not cover it."""
        if version is None or version < self.log_base:
            return None
        return {k for v, k in self.log if v > version}

    def _mut(name):
        base = getattr(dict, name)

        def f(self, *a, **k):
            self.version += 1
            try:
                return base(self, *a, **k)
            finally:
                self.log, self.log_base = [], self.version
        f.__name__ = name
        return f

    for _n in ("update", "pop", "popitem", "clear", "setdefault", "__ior__"):
        locals()[_n] = _mut(_n)
    del _n, _mut


_CACHE_SIZE = 8
_cache = {}  # (id(inserts), dialect, device) -> (inserts, InsertsTable), least recently used first
_dir_snap = {}  # path -> (stat signature, version, {key: value})
_dir_checked = {}  # path -> time.monotonic() of its last signature check
inserts_dir_ttl = 0.0  # seconds a directory signature stays trusted (0: checked on every call)
_dir_bad = {}   # file path -> the error reading it raised (left out of the snapshot)


_LITERAL_KEY = re.compile(r"\{([^{}]*)\}")


def _literal_keys(s):
    """The innermost brace contents of s: the keys it spells out literally (escapes kept)."""
    return _LITERAL_KEY.findall(s)


def _canonical_key(k):
    """The device's rule (ie_device.h missing_status): a key that names a file inside the inserts
    directory (components separated by single '/', none empty, '.' or '..', no NUL); '' is a
    plain miss."""
    if k == "":
        return True
    return "\0" not in k and all(c not in ("", ".", "..") for c in k.split("/"))


def _read_dir_key(key):
    """get_interpdata's file fallback for one key (py:452-461): `<key>.json5` parsed, else `<key>`
    stripped, escaped (recursive_escape on the device); raises FileNotFoundError when neither
    exists, or whatever opening / reading / parsing the file raised."""
    from .program import loads as json5_loads
    try:
        with open(os.path.join(inserts_dir, f"{insertkey_str(key)}.json5")) as f:
            return recursive_escape(json5_loads(f.read()))
    except FileNotFoundError:
        with open(os.path.join(inserts_dir, insertkey_str(key))) as f:
            return recursive_escape(f.read().strip())


def insertkey_str(key):
    return key if isinstance(key, str) else str(key)


def _is_arg_key(k):
    return k.startswith("ARG") and k[3:].isdigit()  # py:437 (str.isdigit: Unicode digits too)


def read_inserts_dir(path):
    """The values get_interpdata's file fallback (py:452-461) finds, before recursive_escape:
    {key: json5.loads(<key>.json5)} or {key: <key> text stripped} for every file under `path`
    (nested files as 'sub/name'; `<key>.json5` first, as py:455-459 tries it first). Keys the
    lookup never sends to the directory ('', 'HH:MM', 'HH:MM:SS', ARGn) are left out."""
    from .program import loads as json5_loads  # the builder's JSON5 reader (json5 is absent here)
    for p in [p for p in _dir_bad if p.startswith(os.path.join(path, ""))]:
        del _dir_bad[p]  # (read again below: a file fixed since reads fine now)
    plain, j5 = {}, {}
    seen = set()
    subdirs = []
    for root, dirs, files in os.walk(path, followlinks=True):  # open() follows links too
        real = os.path.realpath(root)
        if real in seen:  # a link cycle
            dirs[:] = []
            continue
        seen.add(real)
        rel_root = os.path.relpath(root, path)
        for f in files:
            rel = f if rel_root == "." else "/".join(rel_root.split(os.sep) + [f])
            plain[rel] = os.path.join(root, f)
            if rel.endswith(".json5"):
                j5[rel[:-len(".json5")]] = os.path.join(root, f)
        for d in dirs:
            subdirs.append(d if rel_root == "." else "/".join(rel_root.split(os.sep) + [d]))
    # a key naming a subdirectory (and no `<key>.json5` file): py:457 opens the directory, which
    # raises IsADirectoryError when that key is looked up
    for rel in subdirs:
        if rel in j5 or rel in plain:
            continue
        try:
            open(os.path.join(path, rel)).close()
        except OSError as e:
            _dir_bad[os.path.join(path, rel)] = e
    raw = {}
    for key in sorted(set(plain) | set(j5)):
        if key in ("", "HH:MM", "HH:MM:SS") or _is_arg_key(key):
            continue
        try:
            if key in j5:  # py:455-456
                with open(j5[key]) as fh:
                    raw[key] = json5_loads(fh.read())
            else:          # py:457-459
                with open(plain[key]) as fh:
                    raw[key] = fh.read().strip()
        except (OSError, UnicodeDecodeError, ValueError) as e:
            # a file the reference could not read either: it raises only when that key is looked
            # up (py:452-461), so one bad file must not break every other lookup; the key stays out
            # of the snapshot (inserts directory: a lookup of it reports a miss here)
            _dir_bad[os.path.join(path, key)] = e
    return raw


def inserts_dir_snapshot(path):
    """(version, {key: recursive_escape(value)}) for read_inserts_dir(path), the escape on the
    device. The reference reads the files at every lookup; here the directory is re-read when its
    stat signature (every entry's path, type, size and modification time) changed since the last
    call, which sees every write that changes a file's mtime or size. Known deviation: a rewrite
    that keeps a file's size AND lands within one mtime tick of the previous write is not seen
    (the reference, which opens the file at every lookup, sees it). The signature costs one stat
    per entry per call; `inserts_dir_ttl` (seconds, default 0: every call) lets a caller with a
    large, rarely written directory skip it for that long after the last check."""
    hit = _dir_snap.get(path)
    now = time.monotonic()
    if hit is not None and inserts_dir_ttl > 0 and now - _dir_checked.get(path, -1e18) < inserts_dir_ttl:
        return hit[1], hit[2]
    sig = _dir_signature(path)
    _dir_checked[path] = now
    if hit is not None and hit[0] == sig:
        return hit[1], hit[2]
    raw = read_inserts_dir(path)
    keys = list(raw)
    snap = dict(zip(keys, recursive_escape([raw[k] for k in keys]))) if keys else {}
    version = 0 if hit is None else hit[1] + (hit[2] != snap)
    _dir_snap[path] = (sig, version, snap)
    return version, snap


def _dir_signature(path):
    """(relative path, is a directory, size, mtime_ns) of every entry under path (links followed,
    as open() does), sorted."""
    out, seen = [], set()
    for root, dirs, files in os.walk(path, followlinks=True):
        real = os.path.realpath(root)
        if real in seen:
            dirs[:] = []
            continue
        seen.add(real)
        for name in dirs + files:
            p = os.path.join(root, name)
            try:
                st = os.stat(p)
            except OSError:
                out.append((p, None))
                continue
            out.append((p, name in dirs, st.st_size, st.st_mtime_ns))
    out.sort(key=lambda x: x[0])
    return tuple(out)


def table_for(inserts, dialect="py", device=0):
    """The device table for this dict: updated in place when a few keys changed
    (ie_table_set_update), rebuilt when many did; a new clock second rewrites the two clock entries
    in place (ie_table_set_clock). At most _CACHE_SIZE tables stay
    alive (the dict is held with its table, so its id cannot be reused while cached). With
    `inserts_dir` set the table also holds the directory's snapshot, after the inserts."""
    now = _dt.datetime.now()
    clock = (now.hour, now.minute, now.second)
    dir_key = None
    if inserts_dir:
        dver, dsnap = inserts_dir_snapshot(inserts_dir)
        dir_key = (inserts_dir, dver)
    key = (id(inserts), dialect, device)
    hit = _cache.pop(key, None)
    t = hit[1] if hit is not None and hit[0] is inserts else None
    if t is not None and (t.dir_key != dir_key or (not t.matches(inserts) and not (dir_key is None and t.refresh(inserts)))):
        t.close()
        t = None
    if t is not None and t.clock != clock and not t.set_clock(clock):
        t.close()
        t = None
    if t is None:
        extra = {k: v for k, v in dsnap.items() if k not in inserts} if dir_key else None
        t = InsertsTable(inserts, dialect=dialect, clock=clock, device=device, has_inserts_dir=dir_key is not None,
                         extra=extra)
        t.dir_key = dir_key
    _cache[key] = (inserts, t)
    while len(_cache) > _CACHE_SIZE:
        _, old = _cache.pop(next(iter(_cache)))
        old.close()
    return t


def interpolate_states(states, items, dialect="py", device=0):
    """Batch interpolate_inserts over many inserts dicts (forked interpreter states, config 5):
    `items` is a list of (state index, content); one device table set, one batch. Failures are
    returned as exception instances, results in item order."""
    if inserts_dir:  # every state's dict over the directory's snapshot (its own keys win)
        snap = inserts_dir_snapshot(inserts_dir)[1]
        states = [{**snap, **st} for st in states]
    tset = InsertsTableSet(states, dialect=dialect, device=device, has_inserts_dir=bool(inserts_dir))
    try:
        return tset.results([c for _, c in items], [i for i, _ in items])
    finally:
        tset.close()


# ------------------------------------------------------------------------------------------
# the reference surface
# ------------------------------------------------------------------------------------------
def get_interpdata(inserts, insertkey):
    """py:430-467 (host glue for callers' control flow; the device path has it in-kernel)."""
    if insertkey == "HH:MM":
        return _dt.datetime.now().strftime("%H:%M")
    if insertkey == "HH:MM:SS":
        return _dt.datetime.now().strftime("%H:%M:%S")
    if isinstance(insertkey, str) and _is_arg_key(insertkey):
        if insertkey not in inserts:
            raise InterpolationException(
                "Argument interpolation key '%s' is used, but the user passed less than %s program arguments."
                % (insertkey, insertkey[3:]))
        return inserts[insertkey]
    if insertkey == "":
        raise InterpolationException("Tried to interpolate empty string ''.")
    if insertkey in inserts:
        return inserts[insertkey]
    if inserts_dir:  # py:452-461
        try:
            return _read_dir_key(insertkey)
        except FileNotFoundError:
            pass
    detail = " in interpdata" + (" or inserts directory '%s'" % inserts_dir if inserts_dir else "")
    raise InterpolationException("Could not find variable '%s'%s. Available interpolation data keys are %r."
                                 % (insertkey, detail, list(inserts.keys())))


def get_simple_insertkey(content):
    """py:477-495: the key of a whole-string '{...}', '' / None otherwise (same falsy values)."""
    if type(content) != str:
        return None
    if len(content) <= 2:  # the reference's loop, for the tiny cases ('' vs None)
        depth = 0
        for i, c in enumerate(content):
            if c == insert_stop:
                depth -= 1
            if (depth == 0) != (i == 0 or i == len(content) - 1):
                return None
            if c == insert_start:
                depth += 1
        return content[1:-1]
    # (the loop's depth must be non-zero at every inner position: no brace at all fails at the second
    # character; '{key}' with a brace-free key passes; the rest, e.g. 'b}{a' -> '}{', takes the loop)
    if insert_start not in content and insert_stop not in content:
        return None
    inner = content[1:-1]
    if content[0] == insert_start and content[-1] == insert_stop and insert_start not in inner and insert_stop not in inner:
        return inner
    b = N.enc(content)
    o, l = ctypes.c_uint64(), ctypes.c_uint64()
    if N.lib().ie_simple_insertkey(b, len(b), 0, ctypes.byref(o), ctypes.byref(l)):
        return content[1:-1]
    return None


def interpolate_batch(inserts, contents, dialect="py", device=0):
    """Resolve many strings against one inserts snapshot; failures are returned, not raised."""
    return table_for(inserts, dialect, device).results(list(contents))


def interpolate_inserts(inserts, content):
    """py:497-541 — the drop-in. Raises exactly where the reference raises."""
    t = table_for(inserts)
    if type(content) is str:
        r = t.run1(content)
        if r is not _NOT_DONE:
            return r
    r = t.results([content])[0]
    if isinstance(r, BaseException):
        raise r
    return r


def _escape_strings(strings, unescape):
    if not strings:
        return []
    blob, offs = N.pack(strings)
    x = get_exec(0)
    res = ctypes.POINTER(N.BatchRes)()
    bp = ctypes.c_char_p(blob)
    fn = N.lib().ie_unescape_batch if unescape else N.lib().ie_escape_batch
    N.check(fn(x.h, ctypes.cast(bp, ctypes.c_void_p), offs.ctypes.data, len(strings), ctypes.byref(res)),
            "ie_(un)escape_batch")
    outs, _, _ = N.batch_to_python(res)
    return [N.dec(o) for o in outs]


def _map_strings(x, fn_batch):
    """Apply a batched str->str map to every str leaf (list items, dict keys and values)."""
    leaves = []

    def collect(v):
        if type(v) == str:
            leaves.append(v)
        elif type(v) == list:
            for xx in v:
                collect(xx)
        elif type(v) == dict:
            for k, vv in v.items():
                collect(k)
                collect(vv)

    collect(x)
    done = iter(fn_batch(leaves))

    def rebuild(v):
        if type(v) == str:
            return next(done)
        if type(v) == list:
            return [rebuild(xx) for xx in v]
        if type(v) == dict:
            return {rebuild(k): rebuild(vv) for k, vv in v.items()}
        return v

    return rebuild(x)


def recursive_unescape(x):
    """py:1436-1447"""
    return _map_strings(x, lambda ss: _escape_strings(ss, True))


def recursive_escape(x):
    """py:1449-1460"""
    return _map_strings(x, lambda ss: _escape_strings(ss, False))


# ------------------------------------------------------------------------------------------
# ingestion and display sites: the reference's own byte maps on caller text, on
# the device escape / unescape kernels
# ------------------------------------------------------------------------------------------
def ingest_user_inputs(texts):
    """The user_input command's escaping of what the user typed (py:1564-1568: '{' -> '\\{',
    '}' -> '\\}'), for a batch of inputs in one device call."""
    return _escape_strings(list(texts), False)


def ingest_user_input(text):
    return ingest_user_inputs([text])[0]


def ingest_args(args):
    """ARG1, ARG2, ... seeded from the program's command-line arguments, escaped
    (py:2343-2349), one device call: {'ARG1': ..., ...}."""
    return {"ARG%d" % i: v for i, v in enumerate(_escape_strings(list(args), False), start=1)}


def display_texts(texts):
    """The print command's text (py:1669-1673): escaped braces shown as braces, then str(). The
    reference calls .replace before str(), so a non-str text raises AttributeError there and
    here."""
    for t in texts:
        if not isinstance(t, str):
            raise AttributeError("'%s' object has no attribute 'replace'" % type(t).__name__)
    return _escape_strings(list(texts), True)


def display_text(text):
    return display_texts([text])[0]


def unescape_command(inserts, item):
    """The `unescape` command's transform of its item (py:1660-1667): recursive_unescape, then
    recursive_interpolate, which re-enters the result of a whole-string item (py:1463-1464). The
    C ABI's batch form, ie_unescape_cmd_device, reports such items as IE_RECURSE; this is the walk
    its callers do for them."""
    return recursive_interpolate(inserts, recursive_unescape(item))


_LOOP_CMDS = ("for", "serial", "parallel_wait", "parallel_race")


def recursive_interpolate(inserts, x, _depth=0):
    """py:1462-1494 with every string leaf of `x` resolved in one device batch."""
    if _depth > 900:
        raise RecursionError("maximum recursion depth exceeded in recursive_interpolate")
    r = recursive_interpolate_states([inserts], [x], tables=_OneTable(inserts), _depth=_depth)[0]
    if isinstance(r, BaseException):
        raise r
    return r


class _OneTable:
    """table_for(inserts) in the shape recursive_interpolate_states uses (one dict, cached)."""

    def __init__(self, inserts):
        self.t = table_for(inserts)

    def results(self, strings, ids):
        return self.t.results(strings)


def recursive_interpolate_states(states, xs, dialect="py", device=0, tables=None, clock=None, _depth=0):
    """recursive_interpolate (py:1462-1494) of many (state, value) pairs at once: xs[i] is walked
    against states[i] (forked interpreter states, each with its own inserts dict: config 5, the
    per-task pre-pass py:1501 of every state in ONE device batch over a table set; the Rust
    runtime clones the whole map per task instead, rust-project/src/runtime.rs:700-701). Every
    string leaf of every tree goes into the batch; whole-string leaves whose typed result the
    reference walks again (py:1463-1464) go into the next batch, on the same table set. Returns
    one result per pair, or the exception the reference would raise first in that tree's
    traversal order."""
    n = len(states)
    if len(xs) != n:
        raise ValueError("one value per state")
    own = tables is None
    if own:
        tables = InsertsTableSet(states, dialect=dialect, clock=clock, device=device)
    try:
        return _walk_states(states, xs, list(range(n)), tables, _depth)
    finally:
        if own:
            tables.close()


def _walk_states(states, xs, owner, tables, depth):
    """recursive_interpolate of xs[i] against states[owner[i]] (table owner[i] of `tables`)."""
    n = len(xs)
    leaves, ids = [], []
    skels = [None] * n
    fails = [None] * n
    for i in range(n):
        try:
            skels[i] = _tree_leaves(states[owner[i]], xs[i], leaves, ids, owner[i])
        except Exception as e:  # noqa: BLE001 — fails this state only, not the batch
            fails[i] = e
    res = tables.results(leaves, ids) if leaves else []
    # leaves whose result the reference walks again (py:1463-1464): the next batch
    again = [k for k, leaf in enumerate(leaves) if not isinstance(res[k], BaseException) and get_simple_insertkey(leaf)]
    if again:
        if depth >= 900:  # CPython's recursion limit stops the reference
            for k in again:
                res[k] = RecursionError("maximum recursion depth exceeded in recursive_interpolate")
        else:
            sub = _walk_states(states, [res[k] for k in again], [ids[k] for k in again], tables, depth + 1)
            for k, r in zip(again, sub):
                res[k] = r
    out = []
    for i in range(n):
        if fails[i] is not None:
            out.append(fails[i])
            continue
        try:
            out.append(_tree_rebuild(skels[i], res))
        except BaseException as e:  # noqa: BLE001 — the first failing leaf in traversal order
            out.append(e)
    return out


_LEAF = "__ie_leaf__"


def _tree_leaves(inserts, v, leaves, ids, i):
    """The walk of py:1462-1494 without the string work: a skeleton whose str leaves point into
    `leaves` (goto_map / replace_map dicts are kept as they are, py:1471-1477; loop commands get
    their simple `tasks` entries from get_interpdata, py:1479-1489, on the host)."""
    if type(v) == str:
        leaves.append(v)
        ids.append(i)
        return (_LEAF, len(leaves) - 1)
    if type(v) == list:
        return [_tree_leaves(inserts, xx, leaves, ids, i) for xx in v]
    if type(v) == dict:
        cmd = v.get("cmd")
        if cmd in ("goto_map", "replace_map"):  # py:1471-1477
            return (_LEAF + "const", v)
        if cmd in _LOOP_CMDS:  # py:1479-1489
            # a failing lookup is raised where the reference's walk reaches it (_tree_rebuild), so
            # an earlier leaf's error still comes first
            try:
                v = copy.deepcopy(v)
                if (k := get_simple_insertkey(v["tasks"])):
                    v["tasks"] = get_interpdata(inserts, k)
                for j in range(len(v["tasks"])):
                    if (k := get_simple_insertkey(v["tasks"][j])):
                        v["tasks"][j] = get_interpdata(inserts, k)
            except Exception as e:  # noqa: BLE001
                return (_LEAF + "raise", e)
            return (_LEAF + "const", v)
        return (_LEAF + "dict", [(_tree_leaves(inserts, k, leaves, ids, i), _tree_leaves(inserts, vv, leaves, ids, i))
                                 for k, vv in v.items()])
    return (_LEAF + "const", v)


def _tree_rebuild(skel, res):
    if type(skel) == list:
        return [_tree_rebuild(x, res) for x in skel]
    tag, val = skel
    if tag == _LEAF:
        r = res[val]
        if isinstance(r, BaseException):
            raise r
        return r
    if tag == _LEAF + "dict":
        return {_tree_rebuild(k, res): _tree_rebuild(vv, res) for k, vv in val}
    if tag == _LEAF + "raise":
        raise val
    return val
