"""Build an experimental libie_amd variant that differs only in per-source compiler flags:
    python tools/build_flags_variant.py NAME '{"ie_resolve.hip": ["-mllvm", "..."]}'
  -> interpolation-engine_amd/libie_amd_NAME.so (run it with IE_LIB_PATH, tools/gpu_ab.sh NAME)."""
import json
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as G  # noqa: E402


def main():
    name, flags = sys.argv[1], json.loads(sys.argv[2])
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    with tempfile.TemporaryDirectory() as d:
        procs, objs = [], []
        for src in G.SOURCES:
            b = os.path.basename(src)
            obj = os.path.join(d, b + ".o")
            cmd = [hipcc] + G.HIPCC_FLAGS + flags.get(b, []) + ['-DIE_BUILD_ID="variant-%s"' % name, "-c", src, "-o", obj]
            procs.append(subprocess.Popen(cmd, cwd=G.PKG_DIR))
            objs.append(obj)
        if any(p.wait() != 0 for p in procs):
            raise SystemExit("hipcc failed")
        out = os.path.join(G.PKG_DIR, "libie_amd_%s.so" % name)
        subprocess.check_call([hipcc, "--offload-arch=gfx950", "-shared", "-fPIC"] + objs + ["-o", out])
        print(out)


if __name__ == "__main__":
    main()
