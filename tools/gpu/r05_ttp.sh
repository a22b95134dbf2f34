set -o pipefail
D=gpurun_out/r05_ttp
mkdir -p $D
IE_TASK_PROFILE=1 timeout -k 10 300 python -u tools/task_times.py > $D/task_times.json 2> $D/prof.txt
