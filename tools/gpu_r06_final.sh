#!/bin/bash
# Round-6 evidence in one GPU session (TAG names the outputs under gpurun_out/TAG/): smoke, the GPU
# suite, then per config rocprofv3 kernel stats and three PMC passes (FETCH_SIZE, WRITE_SIZE,
# FETCH_SIZE under IE_DEBUG_NOEVAL: tools/pmc_traffic.py's calibrated reads), the traffic file for
# THIS build, one bench line per config (it reads that file), the mirror's latencies, the map-task
# times and the two-rank control plane on one card. Each GPU step under its own limit; the chain
# stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${TAG:-r06f}
O=gpurun_out/$T
mkdir -p $O/traffic
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
if [ -z "${NOTEST:-}" ]; then
  timeout -k 10 240 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
  tail -1 $O/pytest_gpu.log
fi
BID=$(python3 -c "import ctypes; L=ctypes.CDLL('interpolation-engine_amd/libie_amd.so'); L.ie_build_id.restype=ctypes.c_char_p; print(L.ie_build_id().decode())")
for c in ${CONFIGS:-3 2 4 5}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats_cfg$c -o run -- \
    python3 bench.py --config $c --steps 20 --warmup 30 --no-cpu --no-packed --replay 0 > $O/stats_cfg$c.log 2>&1 || { tail -20 $O/stats_cfg$c.log; exit 1; }
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 150 rocprofv3 --pmc $ctr --output-format csv -d $O/pmc_cfg${c}_$ctr -o run -- \
      python3 bench.py --config $c --steps 3 --warmup 1 --no-cpu --no-packed --replay 0 > $O/pmc_cfg${c}_$ctr.log 2>&1 || { tail -20 $O/pmc_cfg${c}_$ctr.log; exit 1; }
  done
  IE_DEBUG_NOEVAL=1 timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_cfg${c}_FETCH_SIZE_noeval -o run -- \
    python3 bench.py --config $c --steps 3 --warmup 1 --no-cpu --no-packed --replay 0 > $O/pmc_cfg${c}_FETCH_SIZE_noeval.log 2>&1 || { tail -20 $O/pmc_cfg${c}_FETCH_SIZE_noeval.log; exit 1; }
  read N S < <(python3 -c "
import json,sys
d=json.loads([l for l in open(sys.argv[1]).read().splitlines() if l.startswith('{')][-1])['config']
n=d['strings_per_gpu']; s=d['input_bytes_per_gpu']+8*(n+1)+(4*n if sys.argv[2]=='5' else 0)
print(n, s)" $O/stats_cfg$c.log $c)
  python3 tools/pmc_traffic.py $c $N $O/pmc_cfg${c}_FETCH_SIZE $O/pmc_cfg${c}_WRITE_SIZE $BID $O/pmc_cfg${c}_FETCH_SIZE_noeval $S || exit 1
  cp profiles/pmc_traffic_cfg$c.json $O/traffic/
  echo "cfg$c profiled"
done
for c in ${CONFIGS:-3 2 4 5}; do
  timeout -k 10 300 python -u bench.py --config $c > $O/bench_cfg$c.log 2>&1 || { tail -20 $O/bench_cfg$c.log; exit 1; }
  tail -1 $O/bench_cfg$c.log | cut -c1-300
done
[ -n "${NOHOST:-}" ] && exit 0
timeout -k 10 300 python -u tools/mirror_latency.py > $O/mirror_latency.json 2> $O/mirror.err || { tail -20 $O/mirror.err; exit 1; }
timeout -k 10 600 python -u tools/task_times.py > $O/task_times.json 2> $O/task_times.err || { tail -20 $O/task_times.err; exit 1; }
timeout -k 10 300 python -u bench.py --gpus 2 --device 0 --steps 10 --warmup 2 --no-cpu > $O/bench_2ranks.log 2>&1 || { tail -20 $O/bench_2ranks.log; exit 1; }
tail -1 $O/bench_2ranks.log
