#!/bin/bash
# One GPU-box session: smoke -> GPU parity tests -> one bench line per config in $CONFIGS
# (default "3 4 5 2") -> optional pipeline-floor experiment (EXP=1). Every GPU step has its own
# time limit and the chain stops at the first failure (no retries).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
TAG=${TAG:-run}
if [ -z "${NOTEST:-}" ]; then
  timeout -k 10 240 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { tail -20 gpurun_out/${TAG}_smoke.log; exit 1; }
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 180 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/${TAG}_pytest_gpu.log 2>&1 || { tail -40 gpurun_out/${TAG}_pytest_gpu.log; exit 1; }
  tail -1 gpurun_out/${TAG}_pytest_gpu.log
fi
for c in ${CONFIGS-3 4 5 2}; do
  timeout -k 10 240 python -u bench.py --config "$c" --steps "${STEPS:-20}" --warmup 3 ${BENCH_ARGS:-} > gpurun_out/${TAG}_bench_cfg$c.log 2>&1 || { tail -20 gpurun_out/${TAG}_bench_cfg$c.log; exit 1; }
  echo "cfg$c $(python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(d['ms_per_step'], r['launch_ms'], r['frac'], (d.get('cpu_baseline') or {}).get('sample','')[-60:])" gpurun_out/${TAG}_bench_cfg$c.log)"
done
if [ -n "${EXP:-}" ]; then
  timeout -k 10 120 ./tools/exp/pipe > gpurun_out/${TAG}_pipe.log 2>&1 || { tail -20 gpurun_out/${TAG}_pipe.log; exit 1; }
  cat gpurun_out/${TAG}_pipe.log
fi
