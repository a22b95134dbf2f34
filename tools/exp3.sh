set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
IE_DEBUG_STAMPS=gpurun_out/stamps.bin timeout -k 10 120 python -u bench.py --steps 2 --warmup 1 --no-cpu > gpurun_out/bench_stamps.log 2>&1 && \
IE_DEBUG_NOEVAL=1 IE_DEBUG_STAMPS=gpurun_out/stamps_noeval.bin timeout -k 10 120 python -u bench.py --steps 2 --warmup 1 --no-cpu > gpurun_out/bench_stamps2.log 2>&1 && \
C="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES" TAGP=pmcA bash tools/gpu_pmc_variants.sh && \
C="SQ_WAVES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT" TAGP=pmcB bash tools/gpu_pmc_variants.sh
