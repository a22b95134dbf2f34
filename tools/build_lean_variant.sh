#!/bin/bash
# Build an experimental libie_amd variant with ie_lean.hip compiled under extra flags:
#   tools/build_lean_variant.sh <name> [hipcc flags, e.g. -DIE_LEAN_WAVES=5 -DIE_LEAN_NT=1]
#     ->  interpolation-engine_amd/libie_amd_<name>.so   (run with IE_LIB_PATH=...)
# The other objects are the main build's (run `g.build()` first).
set -e
cd "$(dirname "$0")/.."
C=interpolation-engine_amd/csrc
O=interpolation-engine_amd/build
name=$1; shift
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wno-unused-result "$@" -c $C/ie_lean.hip -o /tmp/lean_$name.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $O/ie_resolve.hip.o $O/ie_resolve512.hip.o /tmp/lean_$name.o \
  $O/ie_escape.hip.o $O/ie_wildcard.hip.o $O/ie_host.cpp.o -o interpolation-engine_amd/libie_amd_$name.so
