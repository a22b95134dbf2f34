#!/bin/bash
# one rocprofv3 --pmc pass (its counters in $1) over a short config-$CFG bench; summary to stdout
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
TAG=${TAG:-pmc1}
timeout -s KILL 90 rocprofv3 --pmc $1 --output-format csv -d gpurun_out/$TAG -o run -- \
  python3 bench.py --config ${CFG:-3} --steps 3 --warmup 1 --no-cpu > gpurun_out/$TAG.log 2>&1 || { tail -20 gpurun_out/$TAG.log; exit 1; }
python3 tools/pmc_summary.py gpurun_out/$TAG
