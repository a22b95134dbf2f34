#!/bin/bash
# PMC counter passes over a short bench run (each pass its own rocprofv3 --pmc run; no tracing
# domains combined with --pmc). Writes gpurun_out/pmc_<k>/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
rocprofv3 -L > gpurun_out/pmc_list.txt 2>&1 || true
k=0
for set in "$@"; do
  k=$((k+1))
  timeout -k 10 240 rocprofv3 --pmc $set --output-format csv -d gpurun_out/${PFX:-pmc}_$k -o run -- \
    python3 bench.py --steps 3 --warmup 1 --no-cpu ${BENCH_ARGS:-} > gpurun_out/${PFX:-pmc}_$k.log 2>&1 || exit $?
done
