"""Wildcard match / capture on the device (is_wildcard_match / get_wildcard_matches, py:553-567),
the matcher of goto_map, replace_map and delete_except (py:1688-1773; rust-project/src/runtime.rs:
1633-1647, 1754-1775).

  is_wildcard_match(wildcard_s, s)     py:553-555   same name, arguments and result
  get_wildcard_matches(wildcard_s, s)  py:557-567   same name, arguments and result
  Wildcards(patterns).first_match(strings, ranges=None)
      the batch form goto_map / replace_map need: for each string, the first wildcard of the
      (ordered) list that matches it and its captures, all strings in one kernel launch.

Semantics are those of the reference's regex '^' + re.escape(w.replace('*', '〠')).replace('〠',
'(.*)') + '$' under DOTALL (see csrc/ie_wildcard.hip): greedy groups, '$' also before a trailing
newline, a literal U+3020 acting as '*', and a group-less wildcard "capturing" its whole match.
dialect="rs" follows rust-project/src/runtime.rs's regex-crate construction instead ('$' at the
end only, no U+3020 group, no capture without a group; parity unpinned). Every match runs in the
k_wildcard kernel; without libie_amd.so or a GPU these calls raise.
"""
import ctypes

import numpy as np

from . import _native as N


class Wildcards:
    """An ordered list of wildcards compiled onto one device (ie_wildcards_build)."""

    def __init__(self, patterns, device=0, dialect="py"):
        self.patterns = list(patterns)
        self.device = device
        self.dialect = dialect
        blob, offs = N.pack(self.patterns)
        self._blob = blob
        self.h = ctypes.c_void_p()
        bp = ctypes.c_char_p(blob)
        N.check(N.lib().ie_wildcards_build(ctypes.cast(bp, ctypes.c_void_p), offs.ctypes.data, len(self.patterns),
                                           N.IE_DIALECT[dialect], device, ctypes.byref(self.h)), "ie_wildcards_build")

    def close(self):
        if self.h:
            N.lib().ie_wildcards_free(self.h)
            self.h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def match_raw(self, strings, ranges=None, exec_=None):
        """numpy (match[n] int32, ncap[n] uint8, caps[n, IE_WC_MAX_CAP, 2] uint32) for a list of
        str/bytes; ranges: optional [(lo, hi)] per string (the wildcards each string may try)."""
        n = len(strings)
        match = np.full(n, -1, np.int32)
        ncap = np.zeros(n, np.uint8)
        caps = np.zeros((n, N.WC_MAX_CAP, 2), np.uint32)
        if n == 0:
            return match, ncap, caps
        blob, offs = N.pack(strings)
        rng = None if ranges is None else np.ascontiguousarray(np.asarray(ranges, np.uint32).reshape(n, 2))
        from .interpolation_engine import get_exec
        x = exec_ or get_exec(self.device)
        bp = ctypes.c_char_p(blob)
        N.check(N.lib().ie_wildcard_match_batch(x.h, self.h, ctypes.cast(bp, ctypes.c_void_p), offs.ctypes.data, n,
                                                None if rng is None else rng.ctypes.data, match.ctypes.data,
                                                ncap.ctypes.data, caps.ctypes.data), "ie_wildcard_match_batch")
        return match, ncap, caps

    def first_match(self, strings, ranges=None):
        """[(index of the first matching wildcard or -1, [captures as str])] per string."""
        match, ncap, caps = self.match_raw(strings, ranges)
        match, ncap = match.tolist(), ncap.tolist()
        out = []
        for i, s in enumerate(strings):
            if match[i] < 0:
                out.append((-1, []))
                continue
            if not ncap[i]:
                out.append((match[i], []))
                continue
            b = N.enc(s) if isinstance(s, str) else bytes(s)
            out.append((match[i], [N.dec(b[a:a + ln]) for a, ln in caps[i, :ncap[i]].tolist()]))
        return out


_cache = {}


def _single(wildcard_s):
    w = _cache.get(wildcard_s)
    if w is None:
        if len(_cache) > 256:
            _cache.clear()
        w = _cache[wildcard_s] = Wildcards([wildcard_s])
    return w


def is_wildcard_match(wildcard_s, s):
    """py:553-555"""
    return _single(wildcard_s).first_match([s])[0][0] == 0


def get_wildcard_matches(wildcard_s, s):
    """py:557-567: the captures of a matching string (re.findall's groups), [] when it does not match."""
    m, caps = _single(wildcard_s).first_match([s])[0]
    return caps if m == 0 else []
