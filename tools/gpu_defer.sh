#!/bin/bash
# Heavy-string deferral (IE_OPT_DEFER): GPU parity on the views fixtures and the full-size batches,
# then config 5 / 3 / 2 with deferral adaptive (default), off and forced.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
TAG=${TAG:-df}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_programs.py -m gpu -q --maxfail=20 -rf --timeout 300 --timeout-method thread -p no:cacheprovider -k "views or defer or config5 or full" > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; [ $rc -eq 0 ] || [ $rc -eq 1 ] || { tail -30 gpurun_out/${TAG}_pytest.log; exit 1; }
for c in 5 3 2; do
  for d in -1 0 1; do
    IE_DEFER=$d timeout -k 10 150 python -u bench.py --config $c --steps 20 --warmup 5 --no-cpu > gpurun_out/${TAG}_cfg${c}_d$d.log 2>&1 || { tail -20 gpurun_out/${TAG}_cfg${c}_d$d.log; exit 1; }
  done
done
tail -3 gpurun_out/${TAG}_pytest.log
for f in gpurun_out/${TAG}_cfg*.log; do
  echo "$f $(python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(d['ms_per_step'], r['launch_ms'], r['frac'], r['telemetry'])" $f)"
done
