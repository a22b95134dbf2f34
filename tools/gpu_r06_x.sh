set -o pipefail
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/r06_x; mkdir -p $O
export PYTHONUNBUFFERED=1
for r in 1 2; do
  for p in 0 1; do
    IE_PY_PACK=$p timeout -k 10 300 python -u tools/exp/map_phases.py >> $O/map_phases_py$p.jsonl 2>> $O/map_phases.err || { tail -20 $O/map_phases.err; exit 1; }
  done
done
python3 -c "
import json
for p in (0,1):
    for l in open('$O/map_phases_py%d.jsonl'%p):
        d=json.loads(l)['task_step_ms_lib_ms']
        print('py_pack',p,'total',round(sum(r[1] for r in d),1),'lib',round(sum(r[2] for r in d),1),'repl',[r[1] for r in d if r[0]=='repl'])"
