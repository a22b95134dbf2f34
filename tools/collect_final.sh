#!/bin/bash
# Copy one tools/gpu_final.sh run (TAG) from gpurun_out/ into the tracked evidence: DEST (default
# profiles/r03f) gets the bench lines, rocprofv3 kernel stats, GPU test summary, mirror latencies,
# map-task times and the two-rank line; profiles/pmc_traffic_cfgN.json get the run's PMC traffic.
set -e
cd "$(dirname "$0")/.."
T=${1:?TAG}; D=${2:-profiles/r03f}
mkdir -p $D
for c in 2 3 4 5; do
  tail -1 gpurun_out/${T}_bench_cfg$c.log > $D/bench_cfg$c.json
  cp gpurun_out/${T}_stats_cfg$c/run_kernel_stats.csv $D/kernel_stats_cfg$c.csv
  cp gpurun_out/${T}_traffic/pmc_traffic_cfg$c.json profiles/
done
grep -E "passed|failed" gpurun_out/${T}_pytest_gpu.log | tail -1 > $D/pytest_gpu_summary.txt
cp gpurun_out/${T}_mirror.json $D/mirror_latency.json
cp gpurun_out/${T}_task_times.json $D/task_times.json
tail -1 gpurun_out/${T}_bench_2ranks.log > $D/bench_cfg3_2ranks_one_card.json
python3 -c "import json,sys; [json.loads(open(sys.argv[1]+'/bench_cfg%d.json'%c).read()) for c in (2,3,4,5)]" $D
