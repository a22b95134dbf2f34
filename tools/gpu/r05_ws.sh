set -o pipefail
D=gpurun_out/r05_ws
mkdir -p $D
export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $D/ub -o run -- ./tools/exp/store_ubench > $D/ub.txt 2>&1 || exit $?
# config 5's writes split with the diagnostic bits (8: no per-string stores, 4: no stream-out) and
# with the lean first pass off (IE_DEFER=0)
for v in base:0:2 nostores:8:2 nobytes:4:2 nolean:0:0; do
  IFS=: read -r name bits defer <<< "$v"
  IE_DEBUG_NOEVAL=$bits IE_DEFER=$defer timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $D/ws5_$name -o run -- \
    python3 bench.py --steps 3 --warmup 1 --no-cpu --config 5 --replay 0 > $D/ws5_$name.log 2>&1 || exit $?
done
