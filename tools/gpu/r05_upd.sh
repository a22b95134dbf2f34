set -o pipefail
D=gpurun_out/r05_upd
mkdir -p $D
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_table_update.py tests/test_gpu_maps.py > $D/pytest.txt 2>&1 &&
IE_HOST_TRACE=1 timeout -k 10 300 python -u bench.py --config 5 --steps 5 --warmup 2 --no-cpu --replay 4 > $D/bench5.json 2> $D/bench5_trace.txt &&
timeout -k 10 300 python -u bench.py --no-cpu > $D/bench3.json 2> $D/bench3.err
