set -o pipefail
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
bash tools/gpu_ab.sh rb256 rb512 rb256 rb512 || exit 1
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/p12_pytest.log 2>&1 || { tail -40 gpurun_out/p12_pytest.log; exit 1; }
tail -2 gpurun_out/p12_pytest.log
