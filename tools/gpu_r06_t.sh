set -o pipefail
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/r06_t; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u tools/exp/map_phases.py > $O/map_phases.json 2> $O/map_phases.err || { tail -20 $O/map_phases.err; exit 1; }
cat $O/map_phases.json
