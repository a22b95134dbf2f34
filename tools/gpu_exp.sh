#!/bin/bash
# Experiment session: GPU parity tests on the default library, then bench A/B of variant
# libraries (tools/build_variant.sh) and optional PMC passes on the default library.
#   VARIANTS="nott x" PMC="SETS..." bash tools/gpu_exp.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
if [ -z "${NOTEST:-}" ]; then
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
  tail -2 gpurun_out/pytest_gpu.log
fi
for v in base ${VARIANTS:-}; do
  lib=interpolation-engine_amd/libie_amd.so
  [ "$v" != base ] && lib=interpolation-engine_amd/libie_amd_$v.so
  IE_LIB_PATH=$lib timeout -k 10 120 python -u bench.py --steps 20 --warmup 3 --no-cpu ${BENCH_ARGS:-} > gpurun_out/exp_$v.log 2>&1 || { tail -20 gpurun_out/exp_$v.log; exit 1; }
  echo "$v $(python3 -c "import json; d=json.loads(open('gpurun_out/exp_$v.log').read().strip().splitlines()[-1]); r=d['roofline']; print(d['ms_per_step'], r['launch_ms'], r['frac'], r['telemetry'])")"
done
if [ -n "${PMC:-}" ]; then
  cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
  timeout -k 5 60 rocprofv3 -L > gpurun_out/pmc_list.txt 2>&1 || true
  k=0
  for set in $PMC; do
    k=$((k+1))
    timeout -s KILL 90 rocprofv3 --pmc ${set//,/ } --output-format csv -d gpurun_out/pmcx_$k -o run -- \
      python3 bench.py --steps 3 --warmup 1 --no-cpu ${BENCH_ARGS:-} > gpurun_out/pmcx_$k.log 2>&1 || { echo "pmc pass $k failed"; tail -5 gpurun_out/pmcx_$k.log; exit 1; }
  done
fi
