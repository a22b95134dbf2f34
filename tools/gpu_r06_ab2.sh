# config 3 / 2 with the fail-commit evaluator forced on (IE_FAIL_COMMIT=1) against the adaptive
# default (which picks it off: no chain failures), one box, two repetitions
set -o pipefail
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/r06_ab2; mkdir -p $O
export PYTHONUNBUFFERED=1
for r in 1 2; do
  for fc in default 1; do
    for c in 3 2; do
      if [ $fc = default ]; then E=""; else E="IE_FAIL_COMMIT=1"; fi
      env $E timeout -k 10 240 python -u bench.py --config $c --no-cpu --no-packed --replay 0 > $O/bench_fc${fc}_c${c}_r$r.json 2> $O/err.log || { tail -20 $O/err.log; exit 1; }
      python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[2], r['launch_ms'], r['frac'])" $O/bench_fc${fc}_c${c}_r$r.json "fc=$fc cfg$c r$r"
    done
  done
done
