#!/bin/bash
# smoke -> GPU parity tests -> bench (+ variants). Every GPU step has its own time limit; the
# chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 240 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 120 python -u bench.py --steps 10 --warmup 3 --no-cpu > gpurun_out/bench.log 2>&1 && \
IE_DEBUG_NOEVAL=1 timeout -k 10 120 python -u bench.py --steps 10 --warmup 2 --no-cpu > gpurun_out/var_noeval.log 2>&1 && \
IE_DEBUG_STAMPS=gpurun_out/stamps.bin timeout -k 10 120 python -u bench.py --steps 2 --warmup 1 --no-cpu > gpurun_out/bench_stamps.log 2>&1
rc=$?
for f in gpurun_out/bench.log gpurun_out/var_*.log; do [ -f $f ] && echo "$f $(python3 -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['roofline']['launch_ms'], d['roofline']['frac'], d['roofline']['telemetry'])" 2>/dev/null)"; done
exit $rc
