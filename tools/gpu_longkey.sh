#!/bin/bash
# The long-key variant (IE_LONGKEY=1 build): parity on the chain-evaluator tests and config 5's
# full batch, then A/B against the main build on configs 5 and 3.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
IE_LIB_PATH=interpolation-engine_amd/libie_amd_longkey.so timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_programs.py -m gpu -q --maxfail=10 -rf --timeout 300 --timeout-method thread -p no:cacheprovider -k "golden or random or chain or escapes or preresolved or config5 or table" > gpurun_out/lk_pytest.log 2>&1
rc=$?; [ $rc -le 1 ] || { tail -30 gpurun_out/lk_pytest.log; exit 1; }
tail -3 gpurun_out/lk_pytest.log
CONFIGS="5 3" bash tools/gpu_ab2.sh base longkey
