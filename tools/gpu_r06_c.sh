#!/bin/bash
# LEAN5 check: the window / synthetic / full-size GPU tests on the main build, then the A/B benches
# (with one SQ pass each) of VARIANTS
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${TAG:-r06_c}
mkdir -p gpurun_out/$T
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "${PYTEST_K:-window or synthetic or full_size or config or long}" > gpurun_out/$T/pytest.log 2>&1 || { tail -60 gpurun_out/$T/pytest.log; exit 1; }
tail -2 gpurun_out/$T/pytest.log
TAG=$T VARIANTS="${VARIANTS:-main oldlean}" CONFIGS="${CONFIGS:-3 2}" bash tools/gpu_r05_ab.sh
