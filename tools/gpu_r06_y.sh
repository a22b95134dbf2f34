set -o pipefail
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/r06_y; mkdir -p $O
export PYTHONUNBUFFERED=1
PROFILE_TASKS=0,1,3,5 timeout -k 10 300 python -u tools/exp/map_phases.py > $O/map_phases.json 2> $O/profile.txt || { tail -20 $O/profile.txt; exit 1; }
cat $O/map_phases.json
