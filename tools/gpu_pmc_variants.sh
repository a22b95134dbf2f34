#!/bin/bash
# One PMC pass per evaluator variant (diagnostic hooks): pipeline floor, parse, keys, fast, exact.
# Counters from $C (default: instruction mix). No tracing domains are combined with --pmc.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
C=${C:-"SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES"}
TAGP=${TAGP:-pmcv}
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d gpurun_out/${TAGP}_$name -o run -- \
    python3 bench.py --steps 3 --warmup 1 --no-cpu ${BENCH_ARGS:-} > gpurun_out/${TAGP}_$name.log 2>&1
}
run noeval IE_DEBUG_NOEVAL=1 && run fast IE_FAST=1
