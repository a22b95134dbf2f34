set -o pipefail
D=gpurun_out/r05_tt1
mkdir -p $D
IE_TASK_PROFILE_N=1 timeout -k 10 300 python -u tools/task_times.py > $D/task_times.json 2> $D/prof1.txt &&
IE_HOST_TRACE=1 timeout -k 10 300 python -u tools/task_times.py > $D/task_times_tr.json 2> $D/trace.txt
