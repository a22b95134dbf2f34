#!/bin/bash
# Build an experimental libie_amd variant from a (patched) copy of ie_resolve.hip:
#   tools/build_variant.sh <name> <resolve.hip> [extra hipcc flags, e.g. -DIE_EXP_NOEXACT]
#     ->  interpolation-engine_amd/libie_amd_<name>.so
# (run it with IE_LIB_PATH=interpolation-engine_amd/libie_amd_<name>.so)
set -e
cd "$(dirname "$0")/.."
C=interpolation-engine_amd/csrc
name=$1; src=$(readlink -f "$2"); shift 2
tmp=$(mktemp -d)
cp "$src" $tmp/ie_resolve.hip
cp $C/ie_resolve512.hip $tmp/ie_resolve512.hip
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Wno-unused-result -I$C "$@" \
  $tmp/ie_resolve.hip $tmp/ie_resolve512.hip $C/ie_escape.hip $C/ie_wildcard.hip $C/ie_host.cpp -o interpolation-engine_amd/libie_amd_$name.so
rm -rf $tmp
