set -o pipefail
D=gpurun_out/r05_c3ab
mkdir -p $D
for rep in 1 2; do
for r in 32 20 24 48 16; do
  timeout -k 10 240 python -u bench.py --no-cpu --no-packed --reserve $r > $D/res${r}_$rep.json 2> $D/res${r}_$rep.err || exit $?
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print('reserve', sys.argv[2], r['launch_ms'], r['frac'])" $D/res${r}_$rep.json $r
done
IE_LIB_PATH=interpolation-engine_amd/libie_amd_nt0.so timeout -k 10 240 python -u bench.py --no-cpu --no-packed > $D/nt0_$rep.json 2> $D/nt0_$rep.err || exit $?
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print('nt0', r['launch_ms'], r['frac'])" $D/nt0_$rep.json
done
