"""get_interpdata's inserts-directory fallback (py:452-461) against vectors the reference produced
with a real directory (tests/golden/gen_inserts_dir.py): the directory is recreated from the
fixture, read into a snapshot that follows the inserts (the device's view of the lookup order),
and the oracle (CPU) and the device mirror (-m gpu) must reproduce every case."""
import json
import os

import pytest

import __graft_entry__ as G
from oracle import oracle as O
from tests.conftest import ROOT

FIX = json.load(open(os.path.join(ROOT, "tests", "golden", "inserts_dir_py.json"), encoding="utf-8"))


def make_dir(base):
    for rel, text in FIX["files"].items():
        p = os.path.join(base, rel)
        os.makedirs(os.path.dirname(p), exist_ok=True)
        with open(p, "w") as f:
            f.write(text)
    return str(base)


def _escape_tree(v):
    """recursive_escape (py:1449-1460) on the oracle's string escape"""
    if type(v) == str:
        return O.escape(v)
    if type(v) == list:
        return [_escape_tree(x) for x in v]
    if type(v) == dict:
        return {_escape_tree(k): _escape_tree(x) for k, x in v.items()}
    return v


def test_oracle_with_directory_snapshot(tmp_path):
    pkg = G.load_package()
    from interpolation_engine_amd import interpolation_engine as M
    raw = M.read_inserts_dir(make_dir(tmp_path))
    merged = {**{k: _escape_tree(v) for k, v in raw.items()}, **FIX["inserts"]}
    ref = O.Oracle(merged, "py", has_dir=True)
    vals = list(merged.values())
    for c in FIX["cases"]:
        st, out, vid = ref.interpolate(c["s"])
        assert st == c["st"], c
        if st == "OK_STR":
            assert out == c["out"], c
        if st == "OK_VALUE":
            assert vals[vid] == c["value"], c
    del pkg


def test_canonical_path_rule():
    """Keys that are not canonical relative file names stay with the host (NEEDS_HOST)."""
    ref = O.Oracle({"a": "A"}, "py", has_dir=True)
    for k, want in [("x", "E_INTERP"), ("sub/x", "E_INTERP"), ("/etc/passwd", "NEEDS_HOST"), ("../x", "NEEDS_HOST"),
                    ("a//b", "NEEDS_HOST"), ("./x", "NEEDS_HOST"), ("x/", "NEEDS_HOST"), ("..", "NEEDS_HOST"),
                    ("ARG1", "E_INTERP")]:
        assert ref.interpolate("{%s}" % k)[0] == want, k


@pytest.mark.gpu
def test_device_mirror_with_inserts_dir(tmp_path):
    pkg = G.load_package()
    from interpolation_engine_amd import interpolation_engine as M
    d = make_dir(tmp_path)
    old = M.inserts_dir
    M.inserts_dir = d
    try:
        for c in FIX["cases"]:
            try:
                r = pkg.interpolate_inserts(dict(FIX["inserts"]), c["s"])
                st = "OK_STR" if c["st"] == "OK_STR" else "OK_VALUE"
                if st == "OK_STR":
                    assert r == c["out"], c
                else:
                    assert c["st"] == "OK_VALUE" and r == c["value"], (c, r)
            except pkg.InterpolationException:
                assert c["st"] == "E_INTERP", c
            except AssertionError as e:
                if c["st"] not in ("E_ASSERT_TYPE", "E_ASSERT_BRACES"):
                    raise AssertionError("%r: %r" % (c, e))
            # the host helper follows the same order
        assert M.get_interpdata(dict(FIX["inserts"]), "count") == 42
        assert M.get_interpdata(dict(FIX["inserts"]), "over") == "from the inserts"
        with pytest.raises(pkg.InterpolationException):
            M.get_interpdata(dict(FIX["inserts"]), "missing")
    finally:
        M.inserts_dir = old


@pytest.mark.gpu
def test_device_mirror_outside_keys_and_bad_files(tmp_path):
    """Keys that are not canonical file names under the directory (the device reports
    IE_NEEDS_HOST and records the key, also one built from looked-up values; the host opens
    os.path.join(inserts_dir, key) as py:452-461 does and the device resolves the string again) and files the reference cannot read (its error is raised when
    the key is looked up), against the reference's own results (gen_inserts_dir.py)."""
    pkg = G.load_package()
    from interpolation_engine_amd import interpolation_engine as M
    d = make_dir(tmp_path / "dir")
    for rel, text in FIX["outside_files"].items():
        os.makedirs(os.path.dirname(os.path.join(tmp_path, rel)), exist_ok=True)
        with open(os.path.join(tmp_path, rel), "w") as f:
            f.write(text)
    for rel, hx in FIX["bad_files"].items():
        with open(os.path.join(d, rel), "wb") as f:
            f.write(bytes.fromhex(hx))
    old = M.inserts_dir
    M.inserts_dir = d
    try:
        for c in FIX["outside_cases"]:
            try:
                r = pkg.interpolate_inserts(dict(FIX["inserts"], **FIX.get("outside_inserts", {})), c["s"])
            except pkg.InterpolationException:
                assert c["st"] == "E_INTERP", c
                continue
            except Exception as e:  # noqa: BLE001
                assert c["st"] == "RAISES" and type(e).__name__ == c["exc"], (c, e)
                continue
            assert c["st"] in ("OK_STR", "OK_VALUE"), (c, r)
            assert r == (c["out"] if c["st"] == "OK_STR" else c["value"]), (c, r)
    finally:
        M.inserts_dir = old


def test_bad_file_stays_out_of_the_snapshot(tmp_path):
    """One unreadable file (not UTF-8, a broken .json5) must not break the other lookups: the
    reference raises only when that key is looked up (py:452-461); the snapshot leaves it out."""
    G.load_package()
    from interpolation_engine_amd import interpolation_engine as M
    d = make_dir(tmp_path)
    with open(os.path.join(d, "binary"), "wb") as f:
        f.write(b"\xff\xfe\x00 not utf-8")
    with open(os.path.join(d, "broken.json5"), "w") as f:
        f.write("{unterminated: ")
    raw = M.read_inserts_dir(d)
    assert "binary" not in raw and "broken" not in raw
    assert raw["count"] == 42
    assert os.path.join(d, "binary") in M._dir_bad and os.path.join(d, "broken") in M._dir_bad


@pytest.mark.gpu
def test_directory_changes_are_seen_at_the_next_call(tmp_path):
    """The reference opens the file at every lookup (py:452-461): a file written, rewritten (same
    size too), added or removed between two calls is what the next call sees."""
    pkg = G.load_package()
    from interpolation_engine_amd import interpolation_engine as M
    d = str(tmp_path)
    p = os.path.join(d, "v")
    old = M.inserts_dir
    M.inserts_dir = d
    try:
        with open(p, "w") as f:
            f.write("one")
        ins = {"name": "Tom"}
        assert pkg.interpolate_inserts(ins, "<{v}>") == "<one>"
        st = os.stat(p)
        with open(p, "w") as f:
            f.write("two")  # same size: the modification time tells
        os.utime(p, ns=(st.st_atime_ns, st.st_mtime_ns + 1_000_000_000))
        assert pkg.interpolate_inserts(ins, "<{v}>") == "<two>"
        with open(os.path.join(d, "w.json5"), "w") as f:
            f.write("'added'")
        assert pkg.interpolate_inserts(ins, "{w}|{v}") == "added|two"
        os.remove(p)
        with pytest.raises(pkg.InterpolationException):
            pkg.interpolate_inserts(ins, "<{v}>")
        os.makedirs(os.path.join(d, "v"))
        with pytest.raises(IsADirectoryError):
            pkg.interpolate_inserts(ins, "<{v}>")
    finally:
        M.inserts_dir = old
