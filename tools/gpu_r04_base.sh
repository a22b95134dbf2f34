#!/bin/bash
# Round 4 first box: the launcher's GPU test (two ranks on device 0), a config-3 bench line and a
# rocprofv3 kernel-stats pass of the current build.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-r04_base}
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_bench_launch.py -m gpu -x -v --timeout 280 --timeout-method thread -p no:cacheprovider > $O/pytest_launch.log 2>&1 && \
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu > $O/bench_cfg3.json 2> $O/bench_cfg3.err && \
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
  python3 bench.py --steps 10 --warmup 2 --no-cpu > $O/prof.log 2>&1
