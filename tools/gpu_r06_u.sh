set -o pipefail
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/r06_u; mkdir -p $O
export PYTHONUNBUFFERED=1
IE_HOST_TRACE=1 timeout -k 10 300 python -u tools/exp/map_phases.py > $O/map_phases.json 2> $O/host_trace.txt || { tail -20 $O/host_trace.txt; exit 1; }
cat $O/map_phases.json
