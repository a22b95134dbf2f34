#!/bin/bash
# Register / scratch / LDS / occupancy of the LEAN k_resolve instances alone (-DIE_EXP_ONLY_LEAN: a
# ~30 s compile instead of the whole file's); extra hipcc flags as arguments (e.g. -DIE_LEAN5=0)
cd "$(dirname "$0")/../interpolation-engine_amd/csrc"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -mllvm -amdgpu-sched-strategy=max-ilp \
  -DIE_EXP_ONLY_LEAN "$@" -Rpass-analysis=kernel-resource-usage -c ie_resolve.hip -o /tmp/resusage_lean.o --offload-device-only 2>&1 |
  grep -E "error|Function Name|VGPRs:|ScratchSize|Occupancy|LDS Size" | grep -A4 "k_resolve\|error" |
  sed -E 's/.*remark: +//; s/ \[-Rpass.*//' | paste - - - - - | sed -E 's/Function Name: _ZN2ie4r\w+9k_resolveI(\w+)EEvNS[^\t]*\t/\1\t/'
