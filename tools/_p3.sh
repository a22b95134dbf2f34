set -o pipefail
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_wildcard.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/p3_pytest.log 2>&1 || { tail -40 gpurun_out/p3_pytest.log; exit 1; }
tail -2 gpurun_out/p3_pytest.log
bash tools/_p2.sh
