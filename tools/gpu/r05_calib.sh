set -o pipefail
D=gpurun_out/r05_calib
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 60 ./tools/exp/store_ubench > $D/plain.txt &&
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $D/ws -o run -- ./tools/exp/store_ubench > $D/ws.txt 2>&1 &&
bash tools/gpu/r05_tt.sh
