set -o pipefail
D=gpurun_out/r05_ttc
mkdir -p $D
for r in 1 2; do
timeout -k 10 300 python -u tools/task_times.py > $D/task_times_$r.json 2> $D/tt_$r.err || exit $?
done
