#!/bin/bash
# Register / scratch / occupancy of the k_resolve instances (no GPU needed): hipcc's
# kernel-resource-usage remarks for ie_resolve.hip (or the file given).
cd "$(dirname "$0")/../interpolation-engine_amd/csrc"
F=${1:-ie_resolve.hip}
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -mllvm -amdgpu-sched-strategy=max-ilp \
  -Rpass-analysis=kernel-resource-usage -c "$F" -o /tmp/resusage.o --offload-device-only 2>&1 |
  grep -E "Function Name|VGPRs:|ScratchSize|Occupancy" | grep -A3 "k_resolve" |
  sed -E 's/.*remark: +//; s/ \[-Rpass.*//' | paste - - - - | sed -E 's/Function Name: _ZN2ie4r\w+9k_resolveI(\w+)EEvNS[^\t]*\t/\1\t/'
