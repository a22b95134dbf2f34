#!/bin/bash
# Build an experimental libie_amd variant from a (patched) copy of ie_resolve.hip:
#   tools/build_variant.sh <name> <resolve.hip> [extra hipcc flags, e.g. -DIE_EXP_NOEXACT]
#     ->  interpolation-engine_amd/libie_amd_<name>.so
# The other objects are the main build's (run `g.build()` first); ie_resolve.hip gets the
# production flags (__graft_entry__.SOURCE_FLAGS). Run it with
# IE_LIB_PATH=interpolation-engine_amd/libie_amd_<name>.so. SCHED=<strategy> replaces the production
# scheduling strategy of ie_resolve.hip (SCHED=none: LLVM's default).
set -e
cd "$(dirname "$0")/.."
C=interpolation-engine_amd/csrc
O=interpolation-engine_amd/build
name=$1; src=$(readlink -f "$2"); shift 2
tmp=$(mktemp -d)
cp "$src" $tmp/ie_resolve.hip
cp $C/*.h $tmp/
H="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wno-unused-result -I$C -I$tmp"
S="-mllvm -amdgpu-sched-strategy=${SCHED:-max-ilp}"; [ "${SCHED:-}" = none ] && S=""
/opt/rocm/bin/hipcc $H $S "$@" -c $tmp/ie_resolve.hip -o $tmp/r.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $tmp/r.o $O/ie_resolve512.hip.o $O/ie_escape.hip.o \
  $O/ie_wildcard.hip.o $O/ie_host.cpp.o $O/ie_maps.cpp.o -o interpolation-engine_amd/libie_amd_$name.so
rm -rf $tmp
