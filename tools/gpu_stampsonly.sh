#!/bin/bash
# one stamped bench run (per-tile phase timestamps) + one plain bench run
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 120 python -u bench.py --steps 10 --warmup 3 --no-cpu ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1 && \
IE_DEBUG_STAMPS=gpurun_out/stamps.bin timeout -k 10 120 python -u bench.py --steps 2 --warmup 1 --no-cpu ${BENCH_ARGS:-} > gpurun_out/bench_stamps.log 2>&1
rc=$?
python3 -c "import json; d=json.loads(open('gpurun_out/bench.log').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['roofline']['launch_ms'], d['roofline']['frac'])"
exit $rc
