set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
B="timeout -k 10 120 python -u bench.py --steps 10 --warmup 2 --no-cpu"
IE_DEBUG_NOEVAL=1 IE_DEBUG_STAMPS=gpurun_out/st_noeval.bin timeout -k 10 120 python -u bench.py --steps 2 --warmup 1 --no-cpu > gpurun_out/e_st_noeval.log 2>&1 && \
IE_LIB_PATH=$PWD/interpolation-engine_amd/libie_amd_noticket.so IE_DEBUG_NOEVAL=1 $B > gpurun_out/e_nt_noeval.log 2>&1 && \
IE_LIB_PATH=$PWD/interpolation-engine_amd/libie_amd_noticket.so $B > gpurun_out/e_nt_fast.log 2>&1 && \
IE_LIB_PATH=$PWD/interpolation-engine_amd/libie_amd_noticket.so IE_DEBUG_NOEVAL=1 IE_DEBUG_STAMPS=gpurun_out/st_nt_noeval.bin timeout -k 10 120 python -u bench.py --steps 2 --warmup 1 --no-cpu > gpurun_out/e_st_nt_noeval.log 2>&1
for f in gpurun_out/e_nt*.log; do echo "$f $(python3 -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['roofline']['launch_ms'])")"; done
