#!/bin/bash
# A/B of experimental library builds (tools/build_variant.sh): bench per variant and config
# (CONFIGS, default "3"), plus the pipeline floor (IE_DEBUG_NOEVAL) unless NOFLOOR is set.
#   CONFIGS="3 2" bash tools/gpu_ab.sh base vA vB
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for v in "$@"; do
  for c in ${CONFIGS:-3}; do
    IE_LIB_PATH=interpolation-engine_amd/libie_amd_$v.so timeout -k 10 120 python -u bench.py --config $c --steps 20 --warmup 3 --no-cpu > gpurun_out/ab_${v}_cfg$c.log 2>&1 || exit $?
  done
  if [ -z "${NOFLOOR:-}" ]; then
    IE_DEBUG_NOEVAL=1 IE_LIB_PATH=interpolation-engine_amd/libie_amd_$v.so timeout -k 10 120 python -u bench.py --steps 10 --warmup 2 --no-cpu > gpurun_out/ab_${v}_noeval.log 2>&1 || exit $?
  fi
done
for v in "$@"; do for f in gpurun_out/ab_${v}_cfg*.log gpurun_out/ab_${v}_noeval.log; do
  if [ -f "$f" ]; then echo "$f $(python3 -c "import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); r=d['roofline']; print(d['ms_per_step'], r['launch_ms'], r['frac'], r.get('telemetry',{}).get('windowed_tiles'))")"; fi; done; done
