#!/bin/bash
# k_lean (views batches): GPU parity on the views fixtures and the full-size batches, then the bench
# with and without it (IE_LEAN=0). Each step under its own time limit, chained with &&.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
TAG=${TAG:-lean}
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -m gpu -q --maxfail=30 -rf --timeout 120 --timeout-method thread -p no:cacheprovider -k "views" > gpurun_out/${TAG}_pytest_views.log 2>&1
rc=$?; [ $rc -eq 0 ] || [ $rc -eq 1 ] || { tail -30 gpurun_out/${TAG}_pytest_views.log; exit 1; }  # test failures: go on
timeout -k 10 400 python -u -m pytest tests/test_gpu_fullsize.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_pytest_full.log 2>&1
rc=$?; [ $rc -eq 0 ] || [ $rc -eq 1 ] || { tail -30 gpurun_out/${TAG}_pytest_full.log; exit 1; }
for c in ${CONFIGS:-3 2 4 5}; do
  for l in 1 0; do
    IE_LEAN=$l timeout -k 10 150 python -u bench.py --config $c --steps 20 --warmup 3 --no-cpu > gpurun_out/${TAG}_cfg${c}_lean$l.log 2>&1 || { tail -20 gpurun_out/${TAG}_cfg${c}_lean$l.log; exit 1; }
  done
done
for f in gpurun_out/${TAG}_cfg*.log; do
  echo "$f $(python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(d['ms_per_step'], r['launch_ms'], r['frac'])" $f)"
done
tail -2 gpurun_out/${TAG}_pytest_views.log gpurun_out/${TAG}_pytest_full.log
