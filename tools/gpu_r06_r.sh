# where run_map_tasks' host time goes at 10k states (cProfile of the second run)
set -o pipefail
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/r06_r; mkdir -p $O
export PYTHONUNBUFFERED=1
IE_TASK_PROFILE=1 timeout -k 10 400 python -u tools/task_times.py > $O/task_times.json 2> $O/task_profile.txt || { tail -20 $O/task_profile.txt; exit 1; }
cut -c1-200 $O/task_times.json
