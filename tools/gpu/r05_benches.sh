set -o pipefail
D=gpurun_out/r05h
mkdir -p $D
for c in 3 5; do
  timeout -k 10 300 python -u bench.py --config $c > $D/bench_cfg$c.log 2>&1 || exit $?
done
