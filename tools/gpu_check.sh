#!/bin/bash
# One GPU-box session: smoke -> GPU parity tests -> short bench -> (optional) rocprofv3 stats.
# Every GPU step has its own time limit and the chain stops at the first failure (no retries).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
STEPS=${STEPS:-10}
TAG=${TAG:-run}
timeout -k 10 240 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 200 python -u bench.py --steps "$STEPS" --warmup 3 > gpurun_out/bench.log 2>&1 && \
if [ -n "${PROF:-}" ]; then
  cd /tmp && export TMPDIR=/tmp && cd - >/dev/null && \
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$TAG -o run -- \
    python3 bench.py --steps 10 --warmup 2 --no-cpu > gpurun_out/$TAG.log 2>&1
fi
