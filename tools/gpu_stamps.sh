#!/bin/bash
# smoke + GPU tests + a stamped bench run (per-tile phase timestamps) for kernel diagnosis
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 240 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu > gpurun_out/bench.log 2>&1 && \
IE_DEBUG_STAMPS=gpurun_out/stamps.bin timeout -k 10 200 python -u bench.py --steps 2 --warmup 1 --no-cpu > gpurun_out/bench_stamps.log 2>&1
