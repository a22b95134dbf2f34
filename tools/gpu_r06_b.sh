set -o pipefail
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/r06_b
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r06_b/pytest.log 2>&1 || { tail -60 gpurun_out/r06_b/pytest.log; exit 1; }
tail -2 gpurun_out/r06_b/pytest.log
TAG=r06_b VARIANTS="main oldlean l5w4nj2" CONFIGS="3 2" bash tools/gpu_r05_ab.sh
