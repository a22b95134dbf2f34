set -o pipefail
D=gpurun_out/r05_full
mkdir -p $D
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $D/pytest_gpu.txt 2>&1 &&
bash tools/gpu/r05_tt.sh
