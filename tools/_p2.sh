set -o pipefail
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
IE_DEBUG_STAMPS=gpurun_out/p2_stamps.bin timeout -k 10 120 python -u bench.py --steps 2 --warmup 1 --no-cpu > gpurun_out/p2_bench_stamps.log 2>&1 || { tail -20 gpurun_out/p2_bench_stamps.log; exit 1; }
python3 tools/stamps3.py gpurun_out/p2_stamps.bin
