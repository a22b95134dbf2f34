#!/bin/bash
# One PMC pass (instruction mix) per evaluator variant: pipeline floor, fast-path stages, exact path.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
C="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS"
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 240 rocprofv3 --pmc $C --output-format csv -d gpurun_out/pmcv_$name -o run -- \
    python3 bench.py --steps 3 --warmup 1 --no-cpu > gpurun_out/pmcv_$name.log 2>&1
}
run exact IE_FAST=0 && run noeval IE_DEBUG_NOEVAL=1 && run parse IE_FAST=2 && run keys IE_FAST=3 && run fast IE_FAST=1
