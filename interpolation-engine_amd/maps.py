"""goto_map and replace_map over batches of interpreter states, on the device.

The reference runs these two commands one string at a time (py:1689-1773): every interpolation
is an interpolate_inserts call, every wildcard test a Python regex. Here one state or many
forked states are advanced together: each step of the reference's loop is ONE device batch over
every state still running it (interpolations on a table set with one inserts dict per state,
k_resolve; wildcard first-match with captures, k_wildcard), so a task costs a handful of launches
whatever the number of states.

  goto_map(inserts, task)              py:1689-1711 for one state (returns what execute_task
                                       returns: {'goto_target': t} or None)
  replace_map(inserts, task)           py:1713-1773 for one state (sets inserts[output_name])
  goto_map_states(states, task)        the same over many states: a list of results, an
  replace_map_states(states, task)     exception instance where the reference would raise

Semantics kept from the reference, step by step:
  goto_map    the text is interpolated first and only InterpolationException is caught
              (py:1692-1696); then every key and every value is interpolated and str()-ed
              (py:1698-1699, errors propagate); on an interpolation error the 'NULL' key's value
              is the target (py:1702-1705), else the first key that wildcard-matches the text.
  replace_map output_name is interpolated (py:1715); recursive_replace walks the item, resolving
              whole-string keys with get_interpdata (py:1749-1754); each string runs replace_str:
              interpolate, then the first map whose interpolated key matches (keys in order: a
              key that fails to interpolate before any match raises), captures bound as '1', '2',
              ... in `inserts | extra_inserts` to interpolate the value, repeated until nothing
              changes when repeat_until_done (py:1720-1745); an InterpolationException anywhere
              sets the raw 'NULL' value instead (py:1761-1771), or fails the task's assertion.
The map keys are interpolated again on every pass of the loop, as the reference does (py:1728),
with the clock re-read (a table set built without a pinned clock); the inserts cannot change
inside the command, so only a clock key read in a key can make two passes differ.
"""
import copy

from . import interpolation_engine as IE
from .wildcard import Wildcards

# a loop that never reaches a fixed point (the reference spins forever): stop and raise
MAX_PASSES = 100000


def _first_key(d):
    return next(iter(d.keys()))


def _first_value(d):
    return next(iter(d.values()))


_WC_CACHE = {}  # compiled pattern lists by (patterns, device, dialect), most recent last
_WC_CACHE_MAX = 64


def _wildcards(pats, device, dialect):
    """The compiled device form of an ordered wildcard list: a map task's keys are the same texts
    call after call (as Python's re caches the reference's compiled regexes), so the last 64 lists
    stay compiled instead of being built and freed for every step."""
    key = (tuple(pats), device, dialect)
    w = _WC_CACHE.pop(key, None)
    if w is None:
        w = Wildcards(pats, device=device, dialect=dialect)
        if len(_WC_CACHE) >= _WC_CACHE_MAX:
            _WC_CACHE.pop(next(iter(_WC_CACHE))).close()
    _WC_CACHE[key] = w
    return w


def _pattern_range(pats, blocks, keys):
    """The [lo, hi) of `keys` in the pattern list `pats`, appended once per distinct key list (the
    map keys are usually the same text in every state)."""
    t = tuple(keys)
    r = blocks.get(t)
    if r is None:
        r = blocks[t] = (len(pats), len(pats) + len(t))
        pats.extend(t)
    return r


def _str_results(tset, strings, ids):
    """interpolate_inserts on the device, then str() (py:1692, 1698-1699, 1722, 1738)."""
    if not len(strings):
        return []
    return [r if isinstance(r, BaseException) else str(r) for r in tset.results(strings, ids)]


# ------------------------------------------------------------------------------------------
# goto_map (py:1689-1711)
# ------------------------------------------------------------------------------------------
def _goto_map_states_host(states, task, dialect="py", device=0, tables=None):
    """goto_map for each state, driven from Python around one device batch per step (the
    inserts-directory path: its keys may need host completion). [{'goto_target': t} | None |
    exception instance]. tables: an
    InsertsTableSet of exactly these states' dicts, to share between tasks that do not change them
    (run_map_tasks does); else one is built for this task."""
    maps = task["target_maps"]
    n, m = len(states), len(maps)
    out = [None] * n
    if n == 0:
        return out
    tset = tables or IE.InsertsTableSet(states, dialect=dialect, device=device)
    try:
        # value text, then all keys, then all values, for every state in one batch
        block = [task["text"]] + [_first_key(d) for d in maps] + [_first_value(d) for d in maps]
        import numpy as np
        res = _str_results(tset, block * n, np.repeat(np.arange(n, dtype=np.uint32), 1 + 2 * m))
    finally:
        if tables is None:
            tset.close()
    texts, keys, vals = [], [], []
    for s in range(n):
        r = res[s * (1 + 2 * m):(s + 1) * (1 + 2 * m)]
        texts.append(r[0])
        keys.append(r[1:1 + m])
        vals.append(r[1 + m:])
    # every matching test of every state in one launch: state s tries its keys (states whose
    # interpolated keys are the same share one block of patterns)
    pending, pats, ranges, blocks = [], [], [], {}
    for s in range(n):
        t = texts[s]
        if isinstance(t, BaseException) and not isinstance(t, IE.InterpolationException):
            out[s] = t  # py:1693 catches InterpolationException only
            continue
        bad = next((x for x in keys[s] + vals[s] if isinstance(x, BaseException)), None)
        if bad is not None:  # py:1698-1699 propagate
            out[s] = bad
            continue
        if isinstance(t, IE.InterpolationException):  # py:1702-1705
            if "NULL" not in keys[s]:
                out[s] = AssertionError("Order Index %s: value text '%s' could not be resolved but 'NULL' is not "
                                        "a key in target_maps." % (task.get("traceback_label"), task["text"]))
                continue
            target = vals[s][keys[s].index("NULL")]
            out[s] = {"goto_target": target} if target != "CONTINUE" else None
            continue
        pending.append(s)
        ranges.append(_pattern_range(pats, blocks, keys[s]))
    if pending:
        found = _wildcards(pats, device, dialect).first_match([texts[s] for s in pending], ranges)
        for s, (r, (p, _)) in zip(pending, zip(ranges, found)):
            if p < 0:  # py:1708
                out[s] = AssertionError("Order Index %s: goto_map has no matches for '%s'."
                                        % (task.get("traceback_label"), texts[s]))
                continue
            target = vals[s][p - r[0]]
            out[s] = {"goto_target": target} if target != "CONTINUE" else None
    return out


def goto_map(inserts, task):
    """py:1689-1711 for one state: {'goto_target': t} or None; raises where the reference raises."""
    r = goto_map_states([inserts], task)[0]
    if isinstance(r, BaseException):
        raise r
    return r


# ------------------------------------------------------------------------------------------
# replace_map (py:1713-1773)
# ------------------------------------------------------------------------------------------
class _Fail(Exception):
    def __init__(self, exc):
        super().__init__(repr(exc))
        self.exc = exc


def _leaves(inserts, x, out):
    """recursive_replace's walk (py:1748-1759) without the string work: whole-string keys are
    resolved with get_interpdata on the host (py:1749-1754); returns a skeleton whose str leaves
    are indices into `out` (the strings replace_str must run on)."""
    if type(x) == str and "{" not in x and "}" not in x:  # (no brace: never a whole-string key, a leaf)
        out.append(x)
        return ("__leaf__", len(out) - 1)
    k = IE.get_simple_insertkey(x)
    if k:
        sub = IE.get_simple_insertkey(k)
        if sub:
            return _leaves(inserts, IE.insert_start + IE.get_interpdata(inserts, sub) + IE.insert_stop, out)
        return _leaves(inserts, IE.get_interpdata(inserts, k), out)
    if type(x) == str:
        out.append(x)
        return ("__leaf__", len(out) - 1)
    if type(x) == list:
        return [_leaves(inserts, xx, out) for xx in x]
    if type(x) == dict:
        return {("__key__", _leaves(inserts, xk, out)): _leaves(inserts, xv, out) for xk, xv in x.items()}
    return x


class _StateDependent(Exception):
    pass


def _static_leaves(x, out):
    """_leaves for an item with no whole-string key anywhere (the walk then reads no state: one
    skeleton and leaf list serve every state); raises _StateDependent otherwise."""
    if type(x) == str and "{" not in x and "}" not in x:
        out.append(x)
        return ("__leaf__", len(out) - 1)
    if IE.get_simple_insertkey(x):
        raise _StateDependent()
    if type(x) == str:
        out.append(x)
        return ("__leaf__", len(out) - 1)
    if type(x) == list:
        return [_static_leaves(xx, out) for xx in x]
    if type(x) == dict:
        return {("__key__", _static_leaves(xk, out)): _static_leaves(xv, out) for xk, xv in x.items()}
    return x


def _rebuild(skel, done):
    if type(skel) == tuple and len(skel) == 2 and skel[0] == "__leaf__":
        return done[skel[1]]
    if type(skel) == list:
        return [_rebuild(x, done) for x in skel]
    if type(skel) == dict:
        return {_rebuild(k[1], done): _rebuild(v, done) for k, v in skel.items()}
    return skel


def _replace_map_states_host(states, task, dialect="py", device=0, tables=None):
    """replace_map for each state, driven from Python (the inserts-directory path). [(output_name,
    value) | exception instance]. The caller
    stores value under output_name (set_interpdata, py:1771-1773); nothing is mutated here.
    tables: as goto_map_states."""
    maps = task["wildcard_maps"]
    n, m = len(states), len(maps)
    repeat = task.get("repeat_until_done", False)
    out = [None] * n
    if n == 0:
        return out
    no_value = object()
    value_if_error = ([_first_value(d) for d in maps if _first_key(d) == "NULL"] + [no_value])[0]  # py:1761
    tset = tables or IE.InsertsTableSet(states, dialect=dialect, device=device)
    try:
        names = tset.results([task["output_name"]] * n, list(range(n)))  # py:1715 (no str(): as the reference)
        keys = _str_results(tset, [_first_key(d) for d in maps] * n, [s for s in range(n) for _ in range(m)])
        # the leaves of every state's item (host walk; a get_interpdata error fails that state)
        skels, leaves, owner = [None] * n, [], []
        for s in range(n):
            if isinstance(names[s], BaseException):
                out[s] = names[s]
                continue
            mine = []
            try:
                skels[s] = _leaves(states[s], task["item"], mine)
            except (IE.InterpolationException, AssertionError, TypeError) as e:
                out[s] = e
                continue
            skels[s] = (skels[s], len(leaves))
            leaves.extend(mine)
            owner.extend([s] * len(mine))
        done, err = _replace_strings(tset, states, leaves, owner, keys, maps, m, repeat, dialect, device)
    finally:
        if tables is None:
            tset.close()
    # per state: the first failing leaf in the reference's traversal order decides (py:1763-1771)
    counts = [0] * n
    for o in owner:
        counts[o] += 1
    for s in range(n):
        if isinstance(names[s], BaseException):
            # output_name is interpolated before the reference's try (py:1715, 1762): its error
            # reaches the caller as it is, whatever 'NULL' says
            out[s] = names[s]
            continue
        if out[s] is not None:
            e = out[s]
        else:
            skel, base = skels[s]
            e = next((err[base + k] for k in range(counts[s]) if err[base + k] is not None), None)
        if e is None:
            out[s] = (names[s], _rebuild(skels[s][0], done[skels[s][1]:]))
        elif isinstance(e, IE.InterpolationException):
            if value_if_error is no_value:  # py:1765-1766
                out[s] = AssertionError("%s: replace_map encountered an interpolation error without 'NULL' key: %r"
                                        % (task.get("traceback_label"), e))
            else:
                out[s] = (names[s], copy.deepcopy(value_if_error))
        else:
            out[s] = e
    return out


def _replace_strings(tset, states, leaves, owner, keys, maps, m, repeat, dialect, device):
    """replace_str (py:1720-1745) on every leaf at once: (results, first error per leaf)."""
    L = len(leaves)
    cur = list(leaves)
    last = list(leaves)
    err = [None] * L
    active = list(range(L))
    vals_raw = [_first_value(d) for d in maps]
    raw_keys = [_first_key(d) for d in maps]
    # the reference interpolates the map keys inside its loop (py:1728): every pass again. They
    # can only differ between passes through the clock keys, so the keys of the first pass are the
    # ones replace_map_states computed; later passes re-read the clock and interpolate them again
    # (in the same batch as the leaves) when some key text holds a brace.
    live_keys = any("{" in k for k in raw_keys)
    pinned = getattr(tset, "clock_pinned", False)
    passes = 0
    while active:
        passes += 1
        if passes > MAX_PASSES:
            for i in active:
                err[i] = RecursionError("replace_map does not reach a fixed point")
            break
        # 1. interpolate (py:1722); the keys of this pass (py:1728)
        batch, ids = [cur[i] for i in active], [owner[i] for i in active]
        kstates = sorted(set(ids)) if passes > 1 and live_keys else []
        if kstates:
            if not pinned:
                now = IE._dt.datetime.now()
                tset.set_clock((now.hour, now.minute, now.second))
            for s in kstates:
                batch.extend(raw_keys)
                ids.extend([s] * m)
        res = _str_results(tset, batch, ids)
        for j, s in enumerate(kstates):
            base = len(active) + j * m
            keys[s * m:(s + 1) * m] = res[base:base + m]
        res = res[:len(active)]
        # per state: the keys before the first key that fails to interpolate (later keys are never
        # tried once one fails: the failure propagates) and that failure
        key_ok, key_err = {}, {}
        for s in set(ids):
            ks = keys[s * m:(s + 1) * m]
            f = next((j for j, k in enumerate(ks) if isinstance(k, BaseException)), m)
            key_ok[s] = f
            key_err[s] = ks[f] if f < m else None
        alive = []
        for i, r in zip(active, res):
            if isinstance(r, BaseException):
                err[i] = r
            else:
                cur[i] = r
                alive.append(i)
        # 2. the first map whose key matches (py:1725-1735), all leaves in one launch
        pats, ranges, tried, blocks = [], [], [], {}
        for i in alive:
            s = owner[i]
            ranges.append(_pattern_range(pats, blocks, keys[s * m:s * m + key_ok[s]]))
            tried.append(i)
        hits = []
        if pats:
            found = _wildcards(pats, device, dialect).first_match([cur[i] for i in tried], ranges)
        else:
            found = [(-1, [])] * len(tried)
        for i, r, (p, caps) in zip(tried, ranges, found):
            if p >= 0:
                hits.append((i, p - r[0], caps))
            elif key_err[owner[i]] is not None:  # a key failed before anything matched
                err[i] = key_err[owner[i]]
        # 3. the matched maps' values against inserts | captures (py:1736-1738), one table per leaf:
        #    the captures and the keys the value can reach (not a copy of the whole state)
        if hits:
            dicts = [_value_dict(states[owner[i]], vals_raw[p], caps, dialect) for i, p, caps in hits]
            xs = IE.InsertsTableSet(dicts, dialect=dialect, device=device)
            try:
                vres = _str_results(xs, [vals_raw[p] for _, p, _ in hits], list(range(len(hits))))
            finally:
                xs.close()
            # a failure's message lists the table's keys (py:467): those again against the whole
            # `inserts | extra_inserts`, so that the text is the reference's
            bad = [j for j, v in enumerate(vres) if isinstance(v, BaseException)]
            if bad:
                full = [dict(states[owner[hits[j][0]]], **{str(k + 1): c for k, c in enumerate(hits[j][2])})
                        for j in bad]
                xs = IE.InsertsTableSet(full, dialect=dialect, device=device)
                try:
                    again = _str_results(xs, [vals_raw[hits[j][1]] for j in bad], list(range(len(bad))))
                finally:
                    xs.close()
                for j, v in zip(bad, again):
                    vres[j] = v
            for (i, _, _), v in zip(hits, vres):
                if isinstance(v, BaseException):
                    err[i] = v
                else:
                    cur[i] = v
        # 4. a fixed point, or one pass without repeat_until_done (py:1742-1745)
        nxt = []
        for i in alive:
            if err[i] is not None:
                continue
            if last[i] == cur[i] or not repeat:
                continue
            last[i] = cur[i]
            nxt.append(i)
        active = nxt
    return cur, err


def _nested(t):
    """does some pair of t hold another '{' (a key built from a lookup: {q-{1}})?"""
    depth = 0
    for c in t:
        if c == "{":
            depth += 1
            if depth > 1:
                return True
        elif c == "}":
            depth = max(depth - 1, 0)
    return False


def _value_dict(state, value, caps, dialect):
    """`inserts | extra_inserts` for interpolating one map value (py:1736-1738), reduced to what the
    interpolation can look up: the captures ('1', '2', ...) and, from the state, the keys the value
    spells out, closed over the keys spelled out by the values they splice (a spliced '{x}' is
    resolved again by the reference's loop). A key built from another lookup ({a-{b}}) cannot be
    known in advance: then the whole state goes in, as in the reference."""
    extra = {str(k + 1): c for k, c in enumerate(caps)}
    if not isinstance(value, str) or _nested(value):
        return dict(state, **extra)
    out, todo, seen = {}, list(IE._literal_keys(value)), set()
    while todo:
        k = todo.pop()
        if k in seen:
            continue
        seen.add(k)
        if k in extra or k not in state:
            continue
        v = state[k]
        out[k] = v
        try:
            text = IE.render(v, dialect)[1]
        except TypeError:
            return dict(state, **extra)
        if "{" in text:
            if _nested(text):
                return dict(state, **extra)
            todo.extend(IE._literal_keys(text))
    out.update(extra)
    return out


# ------------------------------------------------------------------------------------------
# the map commands behind the C ABI (csrc/ie_maps.cpp: ie_goto_map, ie_replace_map, ie_delete_keys)
# ------------------------------------------------------------------------------------------
def _pairs(maps):
    """[(key, value)] of a task's maps, or None when one is not a str (the host-driven path then
    raises where the reference raises)."""
    out = [(_first_key(d), _first_value(d)) for d in maps]
    return out if all(type(k) is str and type(v) is str for k, v in out) else None


def _errors_of(tset, wanted):
    """{(state, string): the exception the reference raises for it}, one device batch."""
    keys = list(dict.fromkeys(wanted))
    got = tset.results([s for _, s in keys], [t for t, _ in keys]) if keys else []
    return {k: (g if isinstance(g, BaseException) else RuntimeError("expected a failure of %r" % (k[1],)))
            for k, g in zip(keys, got)}


def goto_map_states(states, task, dialect="py", device=0, tables=None):
    """goto_map (py:1689-1711) for each state: [{'goto_target': t} | None | exception instance], by
    ONE library call over every state (ie_goto_map: text, keys and values interpolated in one device
    batch, the first match in one k_wildcard launch). tables: an InsertsTableSet of exactly these
    states' dicts, to share between tasks that do not change them (run_map_tasks does); else one is
    built for this task."""
    n = len(states)
    if n == 0:
        return []
    pairs = _pairs(task["target_maps"])
    tset = tables or IE.InsertsTableSet(states, dialect=dialect, device=device)
    try:
        if tset.has_dir or pairs is None or type(task["text"]) is not str:
            return _goto_map_states_host(states, task, dialect, device, tables=tset)
        import ctypes
        arr, keep = IE.N.map_pairs(pairs)
        text = IE.N.enc(task["text"])
        res = ctypes.POINTER(IE.N.MapResult)()
        x = IE.get_exec(tset.device)
        IE.N.check(IE.N.lib().ie_goto_map(x.h, tset.h, text, len(text), arr, len(pairs), ctypes.byref(res)),
                   "ie_goto_map")
        g_text, g_st, g_wh, _, _ = IE.N.map_result_columns(res)
        m = len(pairs)
        src = lambda w: task["text"] if w == 0 else pairs[w - 1][0] if w <= m else pairs[w - 1 - m][1]  # noqa: E731
        OK_STR, E_NO_MATCH, E_NO_NULL = IE.N.OK_STR, IE.N.E_NO_MATCH, IE.N.E_NO_NULL
        errs = _errors_of(tset, [(s, src(g_wh[s])) for s, st in enumerate(g_st)
                                 if st != OK_STR and st != E_NO_MATCH and st != E_NO_NULL])
    finally:
        if tables is None:
            tset.close()
    out = []
    label = task.get("traceback_label")
    for s, st in enumerate(g_st):
        if st == OK_STR:
            target = g_text[s]
            out.append({"goto_target": target} if target != "CONTINUE" else None)
        elif st == E_NO_MATCH:  # py:1708
            out.append(AssertionError("Order Index %s: goto_map has no matches for '%s'." % (label, g_text[s])))
        elif st == E_NO_NULL:  # py:1703
            out.append(AssertionError("Order Index %s: value text '%s' could not be resolved but 'NULL' is not a "
                                      "key in target_maps." % (label, task["text"])))
        else:
            out.append(errs[(s, src(g_wh[s]))])
    return out


def replace_map_states(states, task, dialect="py", device=0, tables=None):
    """replace_map (py:1713-1773) for each state: [(output_name, value) | exception instance]; the
    caller stores value under output_name (set_interpdata, py:1771-1773). The item's walk
    (recursive_replace, py:1748-1759: whole-string keys through get_interpdata) is done here on the
    states' dicts; output_name and every leaf's replace_str loop (interpolate, first matching map,
    the value against inserts | captures, repeat_until_done) are ONE library call over every state
    (ie_replace_map). tables: as goto_map_states."""
    maps = task["wildcard_maps"]
    n, m = len(states), len(maps)
    if n == 0:
        return []
    pairs = _pairs(maps)
    name = task["output_name"]
    tset = tables or IE.InsertsTableSet(states, dialect=dialect, device=device)
    try:
        if tset.has_dir or pairs is None or type(name) is not str:
            return _replace_map_states_host(states, task, dialect, device, tables=tset)
        out = [None] * n
        import ctypes
        import numpy as np
        try:  # an item without whole-string keys: one walk for all states (its leaves repeated)
            lv0 = []
            skel0 = _static_leaves(task["item"], lv0)
        except _StateDependent:
            skel0 = None
        if skel0 is not None:
            k0 = len(lv0)
            skels = [(skel0, s * k0) for s in range(n)]
            leaves = lv0 * n
            owner = [s for s in range(n) for _ in range(k0)]
        else:
            skels, leaves, owner = [None] * n, [], []
            for s in range(n):
                mine = []
                try:
                    skels[s] = (_leaves(states[s], task["item"], mine), len(leaves))
                except (IE.InterpolationException, AssertionError, TypeError) as e:
                    out[s] = e
                    continue
                leaves.extend(mine)
                owner.extend([s] * len(mine))
        arr, keep = IE.N.map_pairs(pairs)
        blob, offs = IE.N.pack(leaves)
        ids = np.asarray(owner, np.uint32)
        nb = IE.N.enc(name)
        res, nres = ctypes.POINTER(IE.N.MapResult)(), ctypes.POINTER(IE.N.MapResult)()
        x = IE.get_exec(tset.device)
        IE.N.check(IE.N.lib().ie_replace_map(x.h, tset.h, nb, len(nb), ctypes.cast(ctypes.c_char_p(blob), ctypes.c_void_p),
                                             offs.ctypes.data, ids.ctypes.data, len(leaves), arr, m,
                                             1 if task.get("repeat_until_done", False) else 0, ctypes.byref(nres),
                                             ctypes.byref(res)), "ie_replace_map")
        OK_STR, OK_VALUE = IE.N.OK_STR, IE.N.OK_VALUE
        n_text, n_st, _, _, n_vid = IE.N.map_result_columns(nres)
        r_text, r_st, r_wh, _, _ = IE.N.map_result_columns(res) if leaves else ([], [], [], [], [])
        # the exceptions of the failed strings (rare): names, leaves, keys; a failed value with the
        # captures its key took (its message lists inserts | extra_inserts, py:467)
        want = [(s, name) for s, st in enumerate(n_st) if st != OK_STR and st != OK_VALUE]
        vfail = []
        for i in [i for i, st in enumerate(r_st) if st != OK_STR]:
            w = r_wh[i]
            if w == 0:
                want.append((owner[i], r_text[i]))
            elif w <= m:
                want.append((owner[i], pairs[w - 1][0]))
            else:
                vfail.append(i)
        errs = _errors_of(tset, want)
        # the interpolated keys whose captures a failed value took
        kwant = list(dict.fromkeys((owner[i], pairs[r_wh[i] - 1 - m][0]) for i in vfail))
        kgot = dict(zip(kwant, _str_results(tset, [k for _, k in kwant], [t for t, _ in kwant])))
    finally:
        if tables is None:
            tset.close()
    # the failed values' exceptions: each value against its state | its captures, all in one table
    # set and one batch (the captures: every failed leaf's text against its interpolated key, one
    # k_wildcard launch)
    verr = {}
    if vfail:
        from .wildcard import Wildcards
        keys_v = [kgot[(owner[i], pairs[r_wh[i] - 1 - m][0])] for i in vfail]
        texts_v = [r_text[i] for i in vfail]
        ok_q = [q for q, k in enumerate(keys_v) if not isinstance(k, BaseException)]
        caps_v = [[] for _ in vfail]
        if ok_q:
            pats = list(dict.fromkeys(keys_v[q] for q in ok_q))
            at = {p: j for j, p in enumerate(pats)}
            wl = Wildcards(pats, device=device, dialect=dialect)
            try:
                got = wl.first_match([texts_v[q] for q in ok_q], [(at[keys_v[q]], at[keys_v[q]] + 1) for q in ok_q])
            finally:
                wl.close()
            for q, (mi, cs) in zip(ok_q, got):
                caps_v[q] = cs if mi >= 0 else []
        fulls = [dict(states[owner[i]], **{str(k + 1): c for k, c in enumerate(caps_v[q])}) for q, i in enumerate(vfail)]
        xs = IE.InsertsTableSet(fulls, dialect=dialect, device=device)
        try:
            got = xs.results([pairs[r_wh[i] - 1 - m][1] for i in vfail], list(range(len(vfail))))
        finally:
            xs.close()
        verr = dict(zip(vfail, got))
    no_value = object()
    value_if_error = ([v for k, v in pairs if k == "NULL"] + [no_value])[0]  # py:1761
    label = task.get("traceback_label")
    if skel0 is not None:
        count = [k0] * n
    else:
        count = [0] * n
        for o in owner:
            count[o] += 1
    for s in range(n):
        st = n_st[s]
        if st != OK_STR and st != OK_VALUE:
            # output_name is interpolated before the reference's try (py:1715, 1762): its error
            # reaches the caller as it is, whatever 'NULL' says
            out[s] = errs[(s, name)]
            continue
        nm = n_text[s] if st == OK_STR else tset.value(n_vid[s])  # (a typed output_name, py:1715)
        if out[s] is not None:
            e = out[s]
        else:
            skel, base = skels[s]
            e, c = None, count[s]
            if r_st[base:base + c].count(OK_STR) == c:  # (every leaf resolved: the common case)
                done = r_text[base:base + c]
            else:
                done = []
                for k in range(base, base + c):
                    if r_st[k] == OK_STR:
                        done.append(r_text[k])
                        continue
                    w = r_wh[k]
                    e = verr[k] if k in verr else errs[(s, r_text[k] if w == 0 else pairs[w - 1][0])]
                    break
        if e is None:
            out[s] = (nm, _rebuild(skel, done))
        elif isinstance(e, IE.InterpolationException):
            if value_if_error is no_value:  # py:1765-1766
                out[s] = AssertionError("%s: replace_map encountered an interpolation error without 'NULL' key: %r"
                                        % (label, e))
            else:
                out[s] = (nm, copy.deepcopy(value_if_error))
        else:
            out[s] = e
    return out


def delete_states(states, task, dialect="py", device=0, tables=None):
    """delete / delete_except (py:1843-1868) in each state: the keys some wildcard matches (delete)
    or no wildcard matches (delete_except) are removed from the state dicts and from `tables` (the
    device copy, ie_delete_keys: every key of every state in one k_wildcard launch). The wildcards
    are the task's after its pre-pass (recursive_interpolate, py:1501): interpolated per state.
    Returns the deleted keys per state."""
    n = len(states)
    if n == 0:
        return []
    except_ = task["cmd"] == "delete_except"
    tset = tables or IE.InsertsTableSet(states, dialect=dialect, device=device, mutable=True)
    out = [[] for _ in range(n)]
    try:
        # the pre-pass on the wildcards (py:1501); states with the same list share one call
        groups = {}
        wl = task["wildcards"]
        if any(IE.get_simple_insertkey(w) or (type(w) is str and "{" in w) for w in wl):
            got = tset.results([w if type(w) is str else str(w) for w in wl] * n,
                               [s for s in range(n) for _ in wl])
            for s in range(n):
                r = got[s * len(wl):(s + 1) * len(wl)]
                bad = next((e for e in r if isinstance(e, BaseException)), None)
                if bad is not None:
                    out[s] = bad
                    continue
                groups.setdefault(tuple(str(v) for v in r), []).append(s)
        else:
            groups[tuple(str(w) for w in wl)] = list(range(n))
        import ctypes
        import numpy as np
        x = IE.get_exec(tset.device)
        for wild, members in groups.items():
            blob, offs = IE.N.pack(list(wild))
            ids = np.asarray(members, np.uint32)
            res = ctypes.POINTER(IE.N.MapResult)()
            IE.N.check(IE.N.lib().ie_delete_keys(x.h, tset.h, ids.ctypes.data, len(members),
                                                 ctypes.cast(ctypes.c_char_p(blob), ctypes.c_void_p), offs.ctypes.data,
                                                 len(wild), 1 if except_ else 0, ctypes.byref(res)), "ie_delete_keys")
            for b, _, s, _, vid in IE.N.map_result_to_python(res):
                k = IE.N.dec(b)
                states[s].pop(k, None)
                out[s].append(k)
                if vid < len(tset.values):  # (the id went back to the table's free list)
                    tset.values[vid] = None
            # keys a dict holds but the table never does (the clock names, ''): the same test
            odd = [(s, k) for s in members for k in states[s] if k in ("", "HH:MM", "HH:MM:SS")]
            if odd:
                from .wildcard import Wildcards
                found = Wildcards(list(wild), device=device, dialect=dialect).first_match([k for _, k in odd])
                for (s, k), (p, _) in zip(odd, found):
                    if (p >= 0) != except_:
                        del states[s][k]
                        out[s].append(k)
    finally:
        if tables is None:
            tset.close()
    return out


REBUILDS = []  # (task, stores, the library's reason) of every table-set rebuild run_map_tasks made


def N_last_error():
    e = IE.N.lib().ie_last_error()
    return e.decode("utf-8", "replace") if e else ""


def run_map_tasks(states, tasks, dialect="py", device=0):
    """goto_map / replace_map / delete / delete_except tasks in order over many states (the
    reference's loop applies them one state at a time): one table set for the whole run, a
    replace_map's results stored into each state (set_interpdata, py:470-471) and a delete's keys
    removed (py:1843-1868) in place on its device copy (ie_table_set_update) before the next task.
    Returns one list of per-state outcomes per task."""
    outs, tset = [], None
    # (the cyclic collector paused for the run: the states' objects are millions, and a full
    # collection in the middle of a step costs tens of ms; the run creates no cycles of its own)
    import gc
    gc_was = gc.isenabled()
    gc.disable()
    try:  # (interpolation_engine._gc_paused's rule, kept inline: the finally also closes the table set)
        for task in tasks:
            if tset is None:
                tset = IE.InsertsTableSet(states, dialect=dialect, device=device, mutable=True)
            if task["cmd"] == "goto_map":
                outs.append(goto_map_states(states, task, dialect, device, tables=tset))
                continue
            if task["cmd"] in ("delete", "delete_except"):
                # (the device copy is updated in place by the library call)
                outs.append(delete_states(states, task, dialect, device, tables=tset))
                continue
            got = replace_map_states(states, task, dialect, device, tables=tset)
            outs.append(got)
            changes = []
            for s, (st, r) in enumerate(zip(states, got)):
                if not isinstance(r, BaseException):
                    st[r[0]] = r[1]  # set_interpdata (py:470-471)
                    changes.append((s, r[0], r[1]))
            # the same stores on the device copy (ie_table_set_update), or a rebuild when a new
            # key found no placement
            if changes and not tset.update(changes):
                REBUILDS.append((task.get("label") or task["cmd"], len(changes), N_last_error()))
                tset.close()
                tset = None
    finally:
        if gc_was:
            gc.enable()
        if tset is not None:
            tset.close()
    return outs


def replace_map(inserts, task):
    """py:1713-1773 for one state: stores the result under the interpolated output_name."""
    r = replace_map_states([inserts], task)[0]
    if isinstance(r, BaseException):
        raise r
    name, value = r
    inserts[name] = value  # set_interpdata (py:470-471)
