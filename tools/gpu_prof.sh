#!/bin/bash
# rocprofv3 kernel trace + stats of a short bench run (no PMC counters in this pass).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
TAG=${TAG:-prof}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$TAG -o run -- \
  python3 bench.py --steps ${STEPS:-5} --warmup 2 --no-cpu ${BENCH_ARGS:-} > gpurun_out/$TAG.log 2>&1
