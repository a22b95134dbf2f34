set -o pipefail
D=gpurun_out/r05_tt
mkdir -p $D
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_table_update.py tests/test_gpu_maps.py > $D/pytest.txt 2>&1 &&
IE_HOST_TRACE=1 timeout -k 10 300 python -u tools/task_times.py > $D/task_times.json 2> $D/tt_trace.txt &&
IE_TASK_PROFILE=1 timeout -k 10 300 python -u tools/task_times.py > $D/task_times2.json 2> $D/prof.txt
