#!/bin/bash
# The whole GPU suite, then config 5 / 3 bench lines and the views claim experiment (config 3).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
TAG=${TAG:-c2}
timeout -k 10 700 python -u -m pytest tests -m gpu -q --maxfail=20 -rf --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_pytest_gpu.log 2>&1
rc=$?; [ $rc -eq 0 ] || [ $rc -eq 1 ] || { tail -30 gpurun_out/${TAG}_pytest_gpu.log; exit 1; }
for c in 5 3; do
  timeout -k 10 150 python -u bench.py --config $c --steps 20 --warmup 3 --no-cpu > gpurun_out/${TAG}_cfg$c.log 2>&1 || { tail -20 gpurun_out/${TAG}_cfg$c.log; exit 1; }
done
TAG=${TAG}_claim CONFIGS=3 bash tools/gpu_claim.sh || exit 1
tail -3 gpurun_out/${TAG}_pytest_gpu.log
for f in gpurun_out/${TAG}_cfg*.log; do
  echo "$f $(python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(d['ms_per_step'], r['launch_ms'], r['frac'], r['telemetry'])" $f)"
done
