#!/bin/bash
# The whole GPU suite on the main build, then base vs prev on configs 3 5 2.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 800 python -u -m pytest tests -m gpu -q --maxfail=10 -rf --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/ab4_pytest.log 2>&1
rc=$?; [ $rc -le 1 ] || { tail -30 gpurun_out/ab4_pytest.log; exit 1; }
tail -3 gpurun_out/ab4_pytest.log
CONFIGS="3 5 2" bash tools/gpu_ab2.sh base prev
