#!/bin/bash
# Round 4 A/B session: LDS microbench, reserved-range parity tests, then for each library in
# LIBS (default: the main build and the variants given) a config-3 bench and one SQ instruction
# PMC pass. Each GPU step under its own time limit; the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-r04_ab}
mkdir -p $O
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
if [ -x tools/exp/lds_ubench ] && [ -z "${NO_UBENCH:-}" ]; then
  timeout -k 10 120 tools/exp/lds_ubench > $O/ubench.txt 2>&1 || exit $?
fi
if [ -n "${PYTEST_K:-}" ]; then
  IE_LIB_PATH=${PYTEST_LIB:-} timeout -k 10 900 python -u -m pytest ${PYTEST_FILES:-tests/test_gpu_parity.py tests/test_gpu_fullsize.py} -m gpu -x -q -k "$PYTEST_K" --timeout 600 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
fi
if [ -n "${PYTEST2_FILES:-}" ]; then
  timeout -k 10 600 python -u -m pytest $PYTEST2_FILES -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest2.log 2>&1 || { tail -30 $O/pytest2.log; exit 1; }
fi
PMC="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY"
for v in ${VARIANTS:-main}; do
  if [ "$v" = main ]; then LIBP=""; else LIBP=interpolation-engine_amd/libie_amd_$v.so; fi
  for args in ${BENCH_SETS:-"--reserve=32"}; do
    a=${args//,/ }
    tag=${v}_$(echo "$args" | tr -c 'a-zA-Z0-9' '_')
    IE_LIB_PATH=$LIBP timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu $a > $O/bench_$tag.json 2> $O/bench_$tag.err || { tail -20 $O/bench_$tag.err; exit 1; }
  done
  if [ -z "${NO_PMC:-}" ]; then
    IE_LIB_PATH=$LIBP timeout -s KILL 90 rocprofv3 --pmc $PMC --output-format csv -d $O/pmc_$v -o run -- \
      python3 bench.py --steps 3 --warmup 1 --no-cpu ${PMC_ARGS:---reserve=32} > $O/pmc_$v.log 2>&1 || exit $?
  fi
done
