set -o pipefail
VARIANTS="main lkj1 main:IE_DEFER=0 lkj1:IE_DEFER=0" CONFIGS=5 REPS="1 2" NO_PMC=1 TAG=r05_lk PYTEST_FILES="tests/test_gpu_fullsize.py tests/test_gpu_table_update.py" bash tools/gpu_r05_ab.sh || exit $?
D=gpurun_out/r05_lk
export TMPDIR=/tmp
for v in lkj1:2 lkj1:0; do
  IFS=: read -r lib defer <<< "$v"
  IE_LIB_PATH=interpolation-engine_amd/libie_amd_$lib.so IE_DEFER=$defer timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $D/ws5_${lib}_d$defer -o run -- \
    python3 bench.py --steps 3 --warmup 1 --no-cpu --config 5 --replay 0 > $D/ws5_${lib}_d$defer.log 2>&1 || exit $?
done
