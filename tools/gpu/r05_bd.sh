set -o pipefail
D=gpurun_out/r05_bd
mkdir -p $D
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > $D/pytest.txt 2>&1 &&
IE_HOST_TRACE=1 timeout -k 10 240 python -u tools/build_profile.py > $D/bp.txt 2> $D/bp_trace.txt &&
timeout -k 10 300 python -u tools/task_times.py > $D/task_times.json 2> $D/tt.err
