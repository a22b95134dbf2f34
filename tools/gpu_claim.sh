#!/bin/bash
# Views output: does the single cursor atomic (one per tile) set the floor? Config 3 (and 2) with
# and without evaluation (IE_DEBUG_NOEVAL bit 0) and with and without the claim (bit 1: each tile
# writes at twice its input offset instead). Each step under its own time limit, chained with &&.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
TAG=${TAG:-claim}
for c in ${CONFIGS:-3 2}; do
  for m in 0 2 1 3; do
    IE_DEBUG_NOEVAL=$m timeout -k 10 120 python -u bench.py --config $c --steps 20 --warmup 3 --no-cpu --layout views > gpurun_out/${TAG}_cfg${c}_m$m.log 2>&1 || { tail -20 gpurun_out/${TAG}_cfg${c}_m$m.log; exit 1; }
  done
done
for f in gpurun_out/${TAG}_*.log; do
  echo "$f $(python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(d['ms_per_step'], r['launch_ms'], r['frac'])" $f)"
done
