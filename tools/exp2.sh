set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
B="timeout -k 10 120 python -u bench.py --steps 10 --warmup 2 --no-cpu"
$B > gpurun_out/e_base.log 2>&1 && IE_DEBUG_NOEVAL=1 $B > gpurun_out/e_base_noeval.log 2>&1 && \
IE_LIB_PATH=$PWD/interpolation-engine_amd/libie_amd_noticket.so $B > gpurun_out/e_nt.log 2>&1 && \
IE_LIB_PATH=$PWD/interpolation-engine_amd/libie_amd_noticket.so IE_DEBUG_NOEVAL=1 $B > gpurun_out/e_nt_noeval.log 2>&1
for f in gpurun_out/e_*.log; do echo "$f $(python3 -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['roofline']['launch_ms'])")"; done
