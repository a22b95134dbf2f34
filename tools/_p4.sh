set -o pipefail
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 180 --timeout-method thread > gpurun_out/p4_pytest.log 2>&1 || { tail -40 gpurun_out/p4_pytest.log; exit 1; }
tail -2 gpurun_out/p4_pytest.log
NOTEST=1 CONFIGS="3 4 5 2" BENCH_ARGS=--no-cpu TAG=p4 bash tools/gpu_all.sh
bash tools/_p2.sh
