#!/bin/bash
# Round evidence in one GPU session (TAG names the outputs): rocprofv3 kernel-trace/stats per
# config, then one PMC pass each for FETCH_SIZE and WRITE_SIZE per config (separate runs, no
# tracing domains with --pmc). The library is built beforehand on the CPU (never under rocprofv3).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
TAG=${TAG:-round}
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for c in ${CONFIGS:-3 2 4 5}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_stats_cfg$c -o run -- \
    python3 bench.py --config $c --steps 10 --warmup 2 --no-cpu > gpurun_out/${TAG}_stats_cfg$c.log 2>&1 || { tail -20 gpurun_out/${TAG}_stats_cfg$c.log; exit 1; }
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d gpurun_out/${TAG}_pmc_cfg${c}_$ctr -o run -- \
      python3 bench.py --config $c --steps 3 --warmup 1 --no-cpu > gpurun_out/${TAG}_pmc_cfg${c}_$ctr.log 2>&1 || { tail -20 gpurun_out/${TAG}_pmc_cfg${c}_$ctr.log; exit 1; }
  done
  echo "cfg$c done"
done
