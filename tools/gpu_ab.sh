#!/bin/bash
# A/B of experimental library builds (tools/build_variant.sh): bench and pipeline-floor per variant.
#   bash tools/gpu_ab.sh base vA vB
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for v in "$@"; do
  IE_LIB_PATH=interpolation-engine_amd/libie_amd_$v.so timeout -k 10 120 python -u bench.py --steps 20 --warmup 3 --no-cpu > gpurun_out/ab_$v.log 2>&1 || exit $?
  IE_DEBUG_NOEVAL=1 IE_LIB_PATH=interpolation-engine_amd/libie_amd_$v.so timeout -k 10 120 python -u bench.py --steps 10 --warmup 2 --no-cpu > gpurun_out/ab_${v}_noeval.log 2>&1 || exit $?
done
for v in "$@"; do for f in gpurun_out/ab_$v.log gpurun_out/ab_${v}_noeval.log; do
  echo "$f $(python3 -c "import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['roofline']['launch_ms'], d['roofline']['frac'])")"; done; done
