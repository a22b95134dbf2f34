#!/bin/bash
# Round 5 A/B session: for each VARIANT (main, or a libie_amd_<v>.so built by build_variant.sh;
# a name starting with "ck" runs with IE_CUCKOO=1, the two-choice table), a config-3 bench (and the
# configs in CONFIGS) and one SQ instruction-count PMC pass; optional GPU test files (PYTEST_FILES)
# per variant. Each GPU step under its own limit; the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-r05_ab}
mkdir -p $O
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
PMC="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY"
for rep in ${REPS:-1}; do
for spec in ${VARIANTS:-main}; do
  # a variant: <library>[:VAR=VALUE,...] (extra environment for its runs); its outputs are named by
  # the spec with ':' ',' '=' turned into '_'
  lib=${spec%%:*}; envs=""; [ "$spec" != "$lib" ] && envs=$(echo "${spec#*:}" | tr ',' ' ')
  v=$(echo "$spec" | tr ':,=' '___')
  if [ "$lib" = main ]; then LIBP=""; else LIBP=interpolation-engine_amd/libie_amd_$lib.so; fi
  CK=0; case $lib in ck*) CK=1;; esac
  if [ -n "${PYTEST_FILES:-}" ] && [ "$rep" = 1 ]; then
    env $envs IE_CUCKOO=$CK IE_LIB_PATH=$LIBP timeout -k 10 600 python -u -m pytest $PYTEST_FILES -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_$v.log 2>&1 || { tail -30 $O/pytest_$v.log; exit 1; }
    tail -1 $O/pytest_$v.log
  fi
  for c in ${CONFIGS:-3}; do
    env $envs IE_CUCKOO=$CK IE_LIB_PATH=$LIBP timeout -k 10 240 python -u bench.py --config $c --steps ${STEPS:-20} --warmup ${WARM:-10} --no-cpu --replay 0 > $O/bench_${v}_c${c}_r$rep.json 2> $O/bench_${v}_c${c}_r$rep.err || { tail -20 $O/bench_${v}_c${c}_r$rep.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[2], d['config']['workload'][:5], r['launch_ms'], r['frac'])" $O/bench_${v}_c${c}_r$rep.json $v
  done
  if [ -z "${NO_PMC:-}" ] && [ "$rep" = 1 ]; then
    env $envs IE_CUCKOO=$CK IE_LIB_PATH=$LIBP timeout -s KILL 90 rocprofv3 --pmc $PMC --output-format csv -d $O/pmc_$v -o run -- \
      python3 bench.py --steps 3 --warmup 1 --no-cpu > $O/pmc_$v.log 2>&1 || exit $?
  fi
done
done
