#!/bin/bash
# k_lean A/B: stamps of the default build, then config 3 (and 2) for each variant library.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
TAG=${TAG:-lab}
IE_DEBUG_STAMPS=gpurun_out/${TAG}_stamps.bin timeout -k 10 120 python -u bench.py --steps 2 --warmup 1 --no-cpu > gpurun_out/${TAG}_stamps.log 2>&1 || { tail -20 gpurun_out/${TAG}_stamps.log; exit 1; }
python3 tools/stamps_lean.py gpurun_out/${TAG}_stamps.bin > gpurun_out/${TAG}_stamps.txt 2>&1
for v in "$@"; do
  for c in ${CONFIGS:-3 2}; do
    lib=interpolation-engine_amd/libie_amd_$v.so; [ "$v" = base ] && lib=interpolation-engine_amd/libie_amd.so
    IE_LIB_PATH=$lib timeout -k 10 120 python -u bench.py --config $c --steps 20 --warmup 3 --no-cpu > gpurun_out/${TAG}_${v}_cfg$c.log 2>&1 || { tail -20 gpurun_out/${TAG}_${v}_cfg$c.log; exit 1; }
  done
done
cat gpurun_out/${TAG}_stamps.txt
for f in gpurun_out/${TAG}_*_cfg*.log; do
  echo "$f $(python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(d['ms_per_step'], r['launch_ms'], r['frac'])" $f)"
done
