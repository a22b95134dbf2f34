#!/bin/bash
# Timing of the evaluator variants (diagnostic hooks): pipeline floor, parse only, keys only,
# full fast path, exact path only; plus a stamped run of the default. One process per variant.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 120 python -u bench.py --steps 10 --warmup 2 --no-cpu ${BENCH_ARGS:-} > gpurun_out/var_$name.log 2>&1
}
run noeval IE_DEBUG_NOEVAL=1 && run parse IE_FAST=2 && run keys IE_FAST=3 && run fast IE_FAST=1 && \
run exact IE_FAST=0 && \
IE_DEBUG_STAMPS=gpurun_out/stamps.bin timeout -k 10 120 python -u bench.py --steps 2 --warmup 1 --no-cpu > gpurun_out/bench_stamps.log 2>&1
for f in gpurun_out/var_*.log; do echo "$f $(python3 -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['roofline']['launch_ms'])")"; done
