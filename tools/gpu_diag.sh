#!/bin/bash
# Diagnostics session: the pipeline-floor experiment (tools/exp/pipe), one stamped config-3 bench
# (per-tile phase times, tools/stamps2.py) and a rocprofv3 kernel trace of a short config-4 bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
TAG=${TAG:-diag}
timeout -k 10 120 ./tools/exp/pipe > gpurun_out/${TAG}_pipe.log 2>&1 || { tail -20 gpurun_out/${TAG}_pipe.log; exit 1; }
cat gpurun_out/${TAG}_pipe.log
IE_DEBUG_STAMPS=gpurun_out/${TAG}_stamps.bin timeout -k 10 120 python -u bench.py --steps 2 --warmup 1 --no-cpu > gpurun_out/${TAG}_bench_stamps.log 2>&1 || { tail -20 gpurun_out/${TAG}_bench_stamps.log; exit 1; }
python3 tools/stamps2.py gpurun_out/${TAG}_stamps.bin
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_cfg4 -o run -- python3 bench.py --config 4 --steps 5 --warmup 2 --no-cpu > gpurun_out/${TAG}_cfg4.log 2>&1 || { tail -20 gpurun_out/${TAG}_cfg4.log; exit 1; }
cat gpurun_out/${TAG}_cfg4/run_kernel_stats.csv | cut -c1-200
