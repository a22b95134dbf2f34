#!/bin/bash
# Per-tile phase stamps (IE_DEBUG_STAMPS) of config 3 in the views layout, with and without
# evaluation; each step under its own limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
TAG=${TAG:-stv}
LAYOUT=${LAYOUT:-views}
IE_DEBUG_STAMPS=gpurun_out/${TAG}_eval.bin timeout -k 10 120 python -u bench.py --steps 2 --warmup 1 --no-cpu --layout $LAYOUT > gpurun_out/${TAG}_eval.log 2>&1 &&
IE_DEBUG_NOEVAL=1 IE_DEBUG_STAMPS=gpurun_out/${TAG}_noeval.bin timeout -k 10 120 python -u bench.py --steps 2 --warmup 1 --no-cpu --layout $LAYOUT > gpurun_out/${TAG}_noeval.log 2>&1
