#!/bin/bash
# base vs prev on configs 3 5 2, config 5 deferred (IE_DEFER=1) on base, and the views parity tests
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
CONFIGS="3 5 2" bash tools/gpu_ab2.sh base prev || exit 1
IE_DEFER=1 timeout -k 10 150 python -u bench.py --config 5 --steps 20 --warmup 3 --no-cpu > gpurun_out/ab3_defer_cfg5.log 2>&1 || { tail -20 gpurun_out/ab3_defer_cfg5.log; exit 1; }
echo "defer cfg5 $(python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(d['ms_per_step'], r['launch_ms'], r['telemetry'])" gpurun_out/ab3_defer_cfg5.log)"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -q --maxfail=10 -rf --timeout 300 --timeout-method thread -p no:cacheprovider -k "views or defer or config5 or long" > gpurun_out/ab3_pytest.log 2>&1
tail -3 gpurun_out/ab3_pytest.log
