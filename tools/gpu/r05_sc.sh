set -o pipefail
D=gpurun_out/r05_sc
mkdir -p $D
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_table_update.py tests/test_gpu_maps.py tests/test_gpu_small_host.py tests/test_gpu_programs.py > $D/pytest.txt 2>&1 &&
timeout -k 10 240 python -u tools/mirror_latency.py > $D/mirror_latency.json 2> $D/mirror_latency.err &&
timeout -k 10 240 python -u tools/scalar_profile.py > $D/scalar_profile.txt 2>&1
