#!/bin/bash
# A/B of library variants on configs (CONFIGS, default "3 2 4"), alternating variants per config
# so that box drift hits both: bench lines under gpurun_out/ab2_<variant>_cfg<c>_<rep>.log
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for c in ${CONFIGS:-3 2 4}; do
  for rep in 1 2; do
    for v in "$@"; do
      lib=interpolation-engine_amd/libie_amd_$v.so; [ "$v" = base ] && lib=interpolation-engine_amd/libie_amd.so
      IE_LIB_PATH=$lib timeout -k 10 150 python -u bench.py --config $c --steps 20 --warmup 3 --no-cpu > gpurun_out/ab2_${v}_cfg${c}_$rep.log 2>&1 || { tail -20 gpurun_out/ab2_${v}_cfg${c}_$rep.log; exit 1; }
    done
  done
done
for f in gpurun_out/ab2_*.log; do
  echo "$f $(python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(d['ms_per_step'], r['launch_ms'], r['frac'])" $f)"
done
