"""Wildcard match / capture (py:553-567): the oracle against the reference-generated vectors
(tests/golden/wildcard_py.jsonl, tests/golden/gen_wildcard.py), a byte-level model of the
kernel's algorithm (rightmost literal placement, csrc/ie_wildcard.hip) against the same vectors,
and (-m gpu) the k_wildcard kernel through the C ABI against both."""
import os
import random

import numpy as np
import pytest

import __graft_entry__ as G
from oracle import oracle as O
from tests.conftest import ROOT, load_golden

GOLDEN = load_golden("wildcard_py.jsonl")


def test_oracle_matches_reference_vectors():
    for r in GOLDEN:
        assert O.is_wildcard_match(r["w"], r["s"]) == r["match"], r
        if r["match"]:
            assert O.get_wildcard_matches(r["w"], r["s"]) == r["caps"], r


def kernel_model(w, s):
    """The kernel's algorithm on UTF-8 bytes: literals split at '*' / U+3020, every literal at its
    rightmost feasible position (right to left), end n preferred over n-1 before a trailing '\\n'."""
    wb, sb = w.encode(), s.encode()
    lits, cur, k = [], b"", 0
    while k < len(wb):
        if wb[k:k + 1] == b"*" or wb[k:k + 3] == "〠".encode():
            lits.append(cur)
            cur = b""
            k += 1 if wb[k:k + 1] == b"*" else 3
        else:
            cur += wb[k:k + 1]
            k += 1
    lits.append(cur)
    n, g = len(sb), len(lits) - 1
    if not sb.startswith(lits[0]):
        return False, []
    ends = [n] + ([n - 1] if sb.endswith(b"\n") else [])
    if g == 0:
        for e in ends:
            if len(lits[0]) == e:
                return True, [lits[0].decode()]
        return False, []
    for e in ends:
        r = e - len(lits[-1])
        if r < len(lits[0]) or sb[r:e] != lits[-1]:
            continue
        pos = {g: r}
        ok = True
        for j in range(g - 1, 0, -1):
            q = sb.rfind(lits[j], len(lits[0]), r)
            if q < 0:
                ok = False
                break
            pos[j] = r = q
        if ok:
            caps = []
            for j in range(1, g + 1):
                a = len(lits[0]) if j == 1 else pos[j - 1] + len(lits[j - 1])
                caps.append(sb[a:pos[j]].decode())
            return True, caps
    return False, []


def test_kernel_algorithm_model_matches_reference_vectors():
    for r in GOLDEN:
        m, caps = kernel_model(r["w"], r["s"])
        assert m == r["match"], r
        if m:
            assert caps == r["caps"], r


def test_kernel_model_random_vs_oracle():
    rng = random.Random(7)
    for _ in range(20000):
        w = "".join(rng.choice("ab*.\n ") for _ in range(rng.randrange(0, 8)))
        s = "".join(rng.choice(["a", "b", ".", "\n", " ", "é"]) for _ in range(rng.randrange(0, 14)))
        m, caps = kernel_model(w, s)
        assert m == O.is_wildcard_match(w, s), (w, s)
        if m:
            assert caps == O.get_wildcard_matches(w, s), (w, s)


# ---------------------------------------------------------------------------------------------
# device
# ---------------------------------------------------------------------------------------------
def _pkg():
    G.build()
    return G.load_package()


@pytest.mark.gpu
def test_device_wildcards_match_reference_vectors():
    """Every golden case in ONE launch: all distinct wildcards compiled once, each string limited
    to its own wildcard through the per-string range."""
    pkg = _pkg()
    pats = sorted({r["w"] for r in GOLDEN})
    idx = {w: i for i, w in enumerate(pats)}
    W = pkg.Wildcards(pats)
    ranges = [(idx[r["w"]], idx[r["w"]] + 1) for r in GOLDEN]
    got = W.first_match([r["s"] for r in GOLDEN], ranges)
    for r, (m, caps) in zip(GOLDEN, got):
        assert (m >= 0) == r["match"], r
        if r["match"]:
            assert m == idx[r["w"]] and caps == r["caps"], (r, caps)
    W.close()


@pytest.mark.gpu
def test_device_first_match_in_list_order():
    """goto_map / replace_map semantics (py:1704, 1735-1742): the first wildcard of the ordered
    list that matches, on the text_adventure.json5 replace_map list."""
    pkg = _pkg()
    maps = ["*<first-output>*</first-output>*", "*<action-output>*</action-output>*",
            "*<query-output>*</query-output>*", "*<query>*</query>*", "*<action>*</action>*", "*  *",
            "*\n\n\n*", "*\n", "\n*", " *", "* ", "*"]
    strings = sorted({r["s"] for r in GOLDEN})
    W = pkg.Wildcards(maps)
    got = W.first_match(strings)
    for s, (m, caps) in zip(strings, got):
        assert (m, caps) == O.first_wildcard_match(maps, s), s
    W.close()


@pytest.mark.gpu
def test_device_long_strings_and_random_vs_oracle():
    """Strings beyond the kernel's LDS stage (2 KB: read from global memory), multibyte text and
    random wildcards, against the oracle."""
    pkg = _pkg()
    rng = random.Random(11)
    words = ["<action>", "</action>", "go", "é€", "😀", "\n", "  ", "north", "x"]
    strings = ["".join(rng.choice(words) for _ in range(rng.randrange(0, 1500))) for _ in range(64)]
    strings += ["".join(rng.choice(["a", "b", "\n", " "]) for _ in range(rng.randrange(0, 30))) for _ in range(3000)]
    pats = ["*<action>*</action>*", "*\n", "*  *", "*", "a*b", "*a*b*", "\n*", "b*\n", "*😀*", "a**a"]
    pats += ["".join(rng.choice("ab*\n ") for _ in range(rng.randrange(0, 6))) for _ in range(30)]
    W = pkg.Wildcards(pats)
    got = W.first_match(strings)
    for s, g in zip(strings, got):
        assert g == O.first_wildcard_match(pats, s), s[:80]
    W.close()


@pytest.mark.gpu
def test_device_rust_dialect_vs_restated_regex():
    """IE_DIALECT_RS: the regex-crate construction of runtime.rs (parity unpinned: no toolchain),
    against its restatement on Python re (\\Z for the crate's '$')."""
    pkg = _pkg()
    rng = random.Random(13)
    pats = ["*", "a*", "*\n", "x〠y", "*|*", "", "ab\n", "*a*b*"] + \
        ["".join(rng.choice("ab*\n 〠") for _ in range(rng.randrange(0, 6))) for _ in range(30)]
    strings = ["", "\n", "ab\n", "x〠y", "a|b"] + \
        ["".join(rng.choice(["a", "b", "\n", " ", "〠"]) for _ in range(rng.randrange(0, 14))) for _ in range(3000)]
    W = pkg.Wildcards(pats, dialect="rs")
    for s, g in zip(strings, W.first_match(strings)):
        assert g == O.first_wildcard_match_rs(pats, s), s
    W.close()
