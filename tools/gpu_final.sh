#!/bin/bash
# Round-end evidence in one GPU session (TAG names the outputs): kernel stats + PMC passes per
# config (gpu_round.sh), the PMC traffic files written for THIS build (copied back under
# gpurun_out/${TAG}_traffic/, since only gpurun_out/ returns), the GPU test suite, one bench line
# per config (they read those traffic files), the mirror's call latencies.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/${TAG:=final}_traffic
export PYTHONUNBUFFERED=1
TAG=$TAG bash tools/gpu_round.sh || exit 1
BID=$(python3 -c "import ctypes; L=ctypes.CDLL('interpolation-engine_amd/libie_amd.so'); L.ie_build_id.restype=ctypes.c_char_p; print(L.ie_build_id().decode())")
for c in ${CONFIGS:-3 2 4 5}; do
  n=$(python3 -c "import json,sys; print(json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])['config']['strings_per_gpu'])" gpurun_out/${TAG}_stats_cfg$c.log 2>/dev/null || echo 0)
  [ "$n" = 0 ] && n=$(grep -o '"strings_per_gpu": [0-9]*' gpurun_out/${TAG}_stats_cfg$c.log | head -1 | grep -o '[0-9]*$')
  python3 tools/pmc_traffic.py $c $n gpurun_out/${TAG}_pmc_cfg${c}_FETCH_SIZE gpurun_out/${TAG}_pmc_cfg${c}_WRITE_SIZE $BID || exit 1
  cp profiles/pmc_traffic_cfg$c.json gpurun_out/${TAG}_traffic/
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 180 --timeout-method thread > gpurun_out/${TAG}_pytest_gpu.log 2>&1 || { tail -40 gpurun_out/${TAG}_pytest_gpu.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest_gpu.log
NOTEST=1 TAG=$TAG bash tools/gpu_all.sh || exit 1
timeout -k 10 300 python -u tools/mirror_latency.py > gpurun_out/${TAG}_mirror.json 2> gpurun_out/${TAG}_mirror.err || { tail -20 gpurun_out/${TAG}_mirror.err; exit 1; }
cat gpurun_out/${TAG}_mirror.json
timeout -k 10 400 python -u tools/task_times.py > gpurun_out/${TAG}_task_times.json 2> gpurun_out/${TAG}_task_times.err || { tail -20 gpurun_out/${TAG}_task_times.err; exit 1; }
cat gpurun_out/${TAG}_task_times.json
# the multi-rank control plane on one card (two ranks on device 0; the 8-GPU curve is the driver's)
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 \
  bench.py --gpus 2 --device 0 --steps 10 --warmup 2 --no-cpu > gpurun_out/${TAG}_bench_2ranks.log 2>&1 || { tail -20 gpurun_out/${TAG}_bench_2ranks.log; exit 1; }
tail -1 gpurun_out/${TAG}_bench_2ranks.log
