#!/bin/bash
# Round 6 session: [pytest -m gpu (PYTEST=1, or the files in PYTEST_FILES)] -> config-3 bench line
# -> the same bench under rocprofv3 --kernel-trace --stats (profile and ms_per_step from ONE run)
# -> the configs in CONFIGS (bench lines, --no-cpu). Each GPU step under its own limit, chained.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-r06}
mkdir -p $O
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
if [ -n "${PYTEST_FILES:-}" ] || [ -n "${PYTEST:-}" ]; then
  timeout -k 10 ${PYTEST_LIMIT:-1100} python -u -m pytest ${PYTEST_FILES:-tests} -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
  tail -2 $O/pytest.log
fi
if [ -z "${NO_BENCH:-}" ]; then
  timeout -k 10 300 python -u bench.py ${BENCH_ARGS:---no-cpu} > $O/bench_cfg3.json 2> $O/bench_cfg3.err || { tail -20 $O/bench_cfg3.err; exit 1; }
  tail -1 $O/bench_cfg3.json
fi
if [ -n "${PROF:-}" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py ${BENCH_ARGS:---no-cpu} > $O/bench_cfg3_prof.json 2> $O/prof.err || { tail -20 $O/prof.err; exit 1; }
  tail -1 $O/bench_cfg3_prof.json
fi
for c in ${CONFIGS:-}; do
  timeout -k 10 300 python -u bench.py --config $c --no-cpu ${CFG_ARGS:-} > $O/bench_cfg$c.json 2> $O/bench_cfg$c.err || { tail -20 $O/bench_cfg$c.err; exit 1; }
  tail -1 $O/bench_cfg$c.json
done
