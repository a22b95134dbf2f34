set -o pipefail
D=gpurun_out/r05_st
mkdir -p $D
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_table_update.py tests/test_gpu_maps.py > $D/pytest.txt 2>&1 || exit $?
for th in 8; do
IE_HOST_TRACE=1 timeout -k 10 300 python -u bench.py --config 5 --steps 5 --warmup 2 --no-cpu --replay 6 > $D/bench5_t$th.json 2> $D/trace_t$th.txt || exit $?
done
