set -o pipefail
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/r06_w; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_maps.py tests/test_gpu_programs.py tests/test_gpu_table_update.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -u tools/exp/map_phases.py > $O/map_phases.json 2> $O/map_phases.err || { tail -20 $O/map_phases.err; exit 1; }
cat $O/map_phases.json
timeout -k 10 400 python -u tools/task_times.py > $O/task_times.json 2> $O/task_times.err || { tail -20 $O/task_times.err; exit 1; }
python3 -c "
import json
d=json.loads(open('$O/task_times.json').read().strip().splitlines()[-1])
print([(k, d[k]['us_per_state_program'], d[k].get('vs_reference')) for k in ('states_1','states_240','states_10000')])"
