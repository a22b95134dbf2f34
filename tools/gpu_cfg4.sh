#!/bin/bash
# Config-4 GPU session: the synthetic-config parity tests, then the config-4 bench (resolve +
# unescape) and the default config-3 bench. Each step has its own limit; the chain stops at a failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread -p no:cacheprovider \
  ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 200 python -u bench.py --config 4 --steps 10 --warmup 3 > gpurun_out/bench_cfg4.log 2>&1 && \
timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu > gpurun_out/bench.log 2>&1
