#!/bin/bash
# Instruction mix of k_resolve (config 3, views) with and without evaluation: one rocprofv3 --pmc
# pass per mode (SQ counters only), each under its own time limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
CTR="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
TAG=${TAG:-pi}
timeout -s KILL 120 rocprofv3 --pmc $CTR --output-format csv -d gpurun_out/${TAG}_eval -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu --layout views ${BENCH_ARGS:-} > gpurun_out/${TAG}_eval.log 2>&1 &&
IE_DEBUG_NOEVAL=1 timeout -s KILL 120 rocprofv3 --pmc $CTR --output-format csv -d gpurun_out/${TAG}_noeval -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu --layout views ${BENCH_ARGS:-} > gpurun_out/${TAG}_noeval.log 2>&1
