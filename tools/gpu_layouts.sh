#!/bin/bash
# A/B of the output layouts on one build: config 3 packed vs views, with and without evaluation
# (IE_DEBUG_NOEVAL: the pipeline floor). Each step under its own time limit, chained with &&.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
TAG=${TAG:-lay}
CFG=${CFG:-3}
for v in packed views; do
  timeout -k 10 120 python -u bench.py --config $CFG --steps 20 --warmup 3 --no-cpu --layout $v > gpurun_out/${TAG}_${v}.log 2>&1 || { tail -20 gpurun_out/${TAG}_${v}.log; exit 1; }
  IE_DEBUG_NOEVAL=1 timeout -k 10 120 python -u bench.py --config $CFG --steps 20 --warmup 3 --no-cpu --layout $v > gpurun_out/${TAG}_${v}_noeval.log 2>&1 || { tail -20 gpurun_out/${TAG}_${v}_noeval.log; exit 1; }
done
for f in gpurun_out/${TAG}_*.log; do
  echo "$f $(python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(d['ms_per_step'], r['launch_ms'], r['frac'])" $f)"
done
