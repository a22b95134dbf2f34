"""The boundary's prototypes, checked three ways without a GPU (VERDICT r2 "fix the boundary and
test prototypes"):
  * the ctypes table of the Python binding (_native.signatures) against include/ie_amd.h,
    parameter by parameter (arity and the scalar/pointer class and width of each argument);
  * the Rust shim of INTEGRATION.md (the `extern "C"` block a maintainer would add to
    rust-project/src) against the same header;
  * a C program compiled with gcc against the header alone (-Wall -Werror, C11) that links
    libie_amd.so and calls every entry point that needs no device.
The library itself is compiled as C++ inside `extern "C"` against the same header, so a definition
that disagreed with its declaration would not compile (C linkage forbids overloads)."""
import ctypes
import os
import re
import subprocess

import pytest

import __graft_entry__ as G
from tests.conftest import ROOT

G.build()
PKG = G.load_package()
N = PKG._native


def header_prototypes():
    """{name: (return type, [parameter types])} from include/ie_amd.h, C types normalised."""
    src = open(os.path.join(ROOT, "include", "ie_amd.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    src = re.sub(r"#[^\n]*", "", src)
    protos = {}
    for m in re.finditer(r"([A-Za-z_][\w \*]*?)\b(ie_[a-z_0-9]+)\s*\(([^;{]*?)\)\s*;", src, flags=re.S):
        ret, name, params = m.group(1), m.group(2), m.group(3)
        ps = [] if params.strip() in ("", "void") else [p.strip() for p in params.split(",")]
        types = []
        for p in ps:
            p = re.sub(r"\s+", " ", p)
            p = re.sub(r"/\*.*?\*/", "", p).strip()
            # drop the parameter name (the last identifier when the declaration has one)
            mm = re.match(r"^(.*?[\s\*])([A-Za-z_]\w*)$", p)
            t = mm.group(1) if mm and mm.group(1).strip() not in ("const", "") else p
            types.append(_norm(t))
        protos[name] = (_norm(ret), types)
    return protos


def _norm(t):
    t = re.sub(r"\s+", " ", t.replace("*", " * ")).strip()
    stars = t.count("*")
    base = t.replace("*", "").replace("const", "").split()
    base = " ".join(b for b in base if b not in ("extern", "struct", "static", "inline"))
    return base + "*" * stars


# a C type -> the classes of ctypes types that may bind it
_SCALARS = {"int": "i32", "int32_t": "i32", "uint32_t": "u32", "uint64_t": "u64", "int64_t": "i64",
            "float": "f32", "void": "void"}


def _ctypes_class(t):
    if t is None:
        return "void"
    if t in (ctypes.c_int, ctypes.c_int32):
        return "i32"
    if t is ctypes.c_uint32:
        return "u32"
    if t is ctypes.c_uint64:
        return "u64"
    if t is ctypes.c_int64:
        return "i64"
    if t is ctypes.c_float:
        return "f32"
    if t in (ctypes.c_void_p, ctypes.c_char_p) or (isinstance(t, type) and issubclass(t, ctypes._Pointer)):
        return "ptr"
    raise AssertionError("unmapped ctypes type %r" % (t,))


def _c_class(t):
    return "ptr" if t.endswith("*") else _SCALARS[t]


def test_header_parses_into_every_export():
    protos = header_prototypes()
    assert sorted(protos) == sorted(N.EXPORTS)


def test_ctypes_table_matches_header_prototypes():
    protos = header_prototypes()
    sig = N.signatures()
    assert sorted(sig) == sorted(protos), set(sig) ^ set(protos)
    bad = []
    for name, (ret, params) in protos.items():
        res, args = sig[name]
        if _ctypes_class(res) != _c_class(ret):
            bad.append((name, "return", ret, res))
        if len(args) != len(params):
            bad.append((name, "arity", len(params), len(args)))
            continue
        for k, (c, py) in enumerate(zip(params, args)):
            if _c_class(c) != _ctypes_class(py):
                bad.append((name, k, c, py))
    assert not bad, bad


_RUST = {"i32": "i32", "u32": "u32", "u64": "u64", "i64": "i64", "c_int": "i32", "f32": "f32"}


def rust_shim_prototypes():
    """{name: (return class, [parameter classes])} from INTEGRATION.md's `extern "C"` block."""
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    blocks = re.findall(r'extern "C" \{(.*?)\n\}', text, flags=re.S)
    assert blocks, "INTEGRATION.md has no extern \"C\" block"
    out = {}
    for b in blocks:
        b = re.sub(r"//[^\n]*", "", b)
        for m in re.finditer(r"pub fn (ie_\w+)\s*\((.*?)\)\s*(?:->\s*([\w:]+))?\s*;", b, flags=re.S):
            name, params, ret = m.group(1), m.group(2), m.group(3)
            cls = []
            for p in [p.strip() for p in params.split(",") if p.strip()]:
                ty = p.split(":", 1)[1].strip()
                cls.append("ptr" if ty.startswith("*") else _RUST[ty])
            out[name] = ("void" if ret is None else _RUST[ret], cls)
    return out


def test_rust_shim_matches_header_prototypes():
    protos = header_prototypes()
    shim = rust_shim_prototypes()
    assert shim, "no prototypes found"
    bad = []
    for name, (ret, params) in shim.items():
        assert name in protos, name
        hret, hparams = protos[name]
        want = [_c_class(t) for t in hparams]
        if ret != _c_class(hret) or params != want:
            bad.append((name, (ret, params), (_c_class(hret), want)))
    assert not bad, bad


C_PROGRAM = r"""
#include <stdio.h>
#include <string.h>
#include "ie_amd.h"

static int fails = 0;
#define CHECK(c) do { if (!(c)) { printf("FAIL %s:%d %s\n", __FILE__, __LINE__, #c); fails++; } } while (0)

int main(void) {
  CHECK(ie_abi_version() == IE_ABI_VERSION);
  CHECK(ie_build_id() != NULL && strlen(ie_build_id()) == 16);
  CHECK(ie_last_error() != NULL);
  CHECK(ie_device_count() >= 0);
  /* get_simple_insertkey (py:477-495) */
  uint64_t ko = 9, kl = 9;
  CHECK(ie_simple_insertkey("{a}", 3, IE_DIALECT_PY, &ko, &kl) == 1 && ko == 1 && kl == 1);
  CHECK(ie_simple_insertkey("{a}/{b}", 7, IE_DIALECT_PY, &ko, &kl) == 0);
  CHECK(ie_simple_insertkey("{}", 2, IE_DIALECT_RS, &ko, &kl) == 1 && kl == 0);
  /* byte-balanced shards (SURVEY 8e) */
  uint64_t offs[5] = {0, 10, 20, 30, 40}, first[3];
  CHECK(ie_shard_bounds(offs, 4, 2, first) == IE_SUCCESS && first[0] == 0 && first[1] == 2 && first[2] == 4);
  CHECK(ie_shard_bounds(NULL, 4, 2, first) == IE_ERR_INVALID);
  /* the synthetic generator (SURVEY 8d) */
  ie_synth* s = NULL;
  CHECK(ie_synth_create(3, 0, &s) == IE_SUCCESS && s != NULL);
  const ie_kv* kv = NULL;
  CHECK(ie_synth_kv(s, &kv) == 100000 && kv != NULL && kv[0].key_len > 0);
  uint64_t so[4], total = 0;
  CHECK(ie_synth_strings_host(s, 0, 3, NULL, 0, so, &total) == IE_SUCCESS && so[3] == total && total >= 3 * 48);
  unsigned char buf[512];
  CHECK(ie_synth_strings_host(s, 0, 3, buf, sizeof buf, so, &total) == IE_SUCCESS);
  CHECK(memchr(buf, '{', total) != NULL);
  ie_synth_free(s);
  CHECK(ie_synth_create(7, 0, &s) == IE_ERR_INVALID);
  /* entry points that need a device refuse cleanly without one (no CPU path) */
  if (ie_device_count() == 0) {
    ie_exec* x = NULL;
    CHECK(ie_exec_create(0, NULL, &x) == IE_ERR_NO_DEVICE);
  }
  printf("%s\n", fails ? "FAILED" : "OK");
  return fails != 0;
}
"""


def test_c_program_against_the_header(tmp_path):
    src = tmp_path / "abi_check.c"
    src.write_text(C_PROGRAM)
    exe = tmp_path / "abi_check"
    libdir = os.path.dirname(N.LIB_PATH)
    cmd = ["gcc", "-std=c11", "-Wall", "-Wextra", "-Werror", "-I", os.path.join(ROOT, "include"), str(src),
           "-L", libdir, "-l:libie_amd.so", "-Wl,-rpath," + libdir, "-Wl,-rpath,/opt/rocm/lib", "-o", str(exe)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and r.stdout.strip().endswith("OK"), r.stdout + r.stderr


def test_rust_shim_constants_match_header():
    """The shim's status and flag constants (its IE_NEEDS_HOST completion branches on them) equal the
    header's enumerators and macros, and the completion's entry point is declared."""
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    consts = {m.group(1): int(m.group(2), 0) for m in re.finditer(r"pub const (IE_\w+): \w+ = (\w+);", text)}
    src = open(os.path.join(ROOT, "include", "ie_amd.h")).read()
    hdr = {m.group(1): int(m.group(2), 0) for m in re.finditer(r"\b(IE_\w+)\s*=\s*(\d+)", src)}
    hdr.update({m.group(1): int(m.group(2), 0) for m in re.finditer(r"#define (IE_\w+) (0x[0-9A-Fa-f]+|\d+)u?\b", src)})
    for name in ("IE_OK_STR", "IE_OK_VALUE", "IE_E_RS_PANIC", "IE_NEEDS_HOST", "IE_TABLE_HAS_INSERTS_DIR",
                 "IE_DIALECT_RS"):
        assert name in consts, name
        assert consts[name] == hdr[name], (name, consts[name], hdr[name])
    assert "ie_exec_host_keys" in rust_shim_prototypes()
