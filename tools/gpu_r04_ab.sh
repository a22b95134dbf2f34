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
# FETCH_SIZE calibration on known byte counts (streaming vs random 64-B entry gathers) and the
# config-4 fetch split (full vs IE_DEBUG_NOEVAL, i.e. without the table lookups)
if [ -n "${GATHER:-}" ]; then
  timeout -k 10 60 tools/exp/gather_ubench > $O/gather.txt 2>&1 || exit $?
  timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/gather_fetch -o run -- tools/exp/gather_ubench > $O/gather_fetch.log 2>&1 || exit $?
  timeout -s KILL 60 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $O/gather_hit -o run -- tools/exp/gather_ubench > $O/gather_hit.log 2>&1 || exit $?
fi
if [ -n "${CFG4_PMC:-}" ]; then
  timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/c4_fetch -o run -- python3 bench.py --config 4 --steps 2 --warmup 1 --no-cpu > $O/c4_fetch.log 2>&1 || exit $?
  IE_DEBUG_NOEVAL=1 timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/c4_fetch_noeval -o run -- python3 bench.py --config 4 --steps 2 --warmup 1 --no-cpu > $O/c4_fetch_noeval.log 2>&1 || exit $?
  timeout -s KILL 150 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $O/c4_hit -o run -- python3 bench.py --config 4 --steps 2 --warmup 1 --no-cpu > $O/c4_hit.log 2>&1 || exit $?
fi
# traffic passes (main build): FETCH_SIZE and WRITE_SIZE, full and IE_DEBUG_NOEVAL (the streaming
# calibration on a known byte count), per config in TRAFFIC_CFGS
for c in ${TRAFFIC_CFGS:-}; do
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 150 rocprofv3 --pmc $ctr --output-format csv -d $O/tr_c${c}_$ctr -o run -- python3 bench.py --config $c --steps 3 --warmup 1 --no-cpu > $O/tr_c${c}_$ctr.log 2>&1 || exit $?
    IE_DEBUG_NOEVAL=1 timeout -s KILL 150 rocprofv3 --pmc $ctr --output-format csv -d $O/tr_c${c}_${ctr}_noeval -o run -- python3 bench.py --config $c --steps 3 --warmup 1 --no-cpu > $O/tr_c${c}_${ctr}_noeval.log 2>&1 || exit $?
  done
done
if [ -n "${PYTEST_ALL:-}" ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -p no:cacheprovider > $O/pytest_all.log 2>&1 || { tail -30 $O/pytest_all.log; exit 1; }
fi
# write split per config in WSPLIT_CFGS: WRITE_SIZE without the byte stream-out (IE_DEBUG_NOEVAL=4)
# and without the per-string stores (=8); with STW set, the status-word variant's full WRITE_SIZE
for c in ${WSPLIT_CFGS:-}; do
  for m in 4 8; do
    IE_DEBUG_NOEVAL=$m timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/ws_c${c}_m$m -o run -- python3 bench.py --config $c --steps 3 --warmup 1 --no-cpu --replay 0 > $O/ws_c${c}_m$m.log 2>&1 || exit $?
  done
  if [ -n "${STW:-}" ]; then
    IE_LIB_PATH=interpolation-engine_amd/libie_amd_$STW.so timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/ws_c${c}_$STW -o run -- python3 bench.py --config $c --steps 3 --warmup 1 --no-cpu > $O/ws_c${c}_$STW.log 2>&1 || exit $?
  fi
done
# the skeleton's instruction counts (IE_DEBUG_NOEVAL=1: stage, classify, build, stream-out only)
if [ -n "${PMC_NOEVAL:-}" ]; then
  IE_DEBUG_NOEVAL=1 timeout -s KILL 90 rocprofv3 --pmc $PMC --output-format csv -d $O/pmc_main_noeval -o run -- \
    python3 bench.py --steps 3 --warmup 1 --no-cpu --reserve=32 > $O/pmc_main_noeval.log 2>&1 || exit $?
fi
# WRITE_SIZE per variant (WRITE_VARIANTS) for the configs in WRITE_CFGS
for v in ${WRITE_VARIANTS:-}; do
  if [ "$v" = main ]; then LIBP=""; else LIBP=interpolation-engine_amd/libie_amd_$v.so; fi
  for c in ${WRITE_CFGS:-5 3}; do
    IE_LIB_PATH=$LIBP timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/wv_${v}_c$c -o run -- python3 bench.py --config $c --steps 3 --warmup 1 --no-cpu --replay 0 > $O/wv_${v}_c$c.log 2>&1 || exit $?
  done
done
