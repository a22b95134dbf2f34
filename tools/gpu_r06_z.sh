# L2 (TCC) hits and misses of config 3's k_resolve, with evaluation and without (IE_DEBUG_NOEVAL):
# the difference is the table lookups' share
set -o pipefail
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/r06_z; mkdir -p $O
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for c in 3 4; do
  timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $O/tcc_cfg$c -o run -- python3 bench.py --config $c --steps 3 --warmup 1 --no-cpu --no-packed --replay 0 > $O/tcc_cfg$c.log 2>&1 || { tail -20 $O/tcc_cfg$c.log; exit 1; }
  IE_DEBUG_NOEVAL=1 timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $O/tcc_cfg${c}_noeval -o run -- python3 bench.py --config $c --steps 3 --warmup 1 --no-cpu --no-packed --replay 0 > $O/tcc_cfg${c}_noeval.log 2>&1 || { tail -20 $O/tcc_cfg${c}_noeval.log; exit 1; }
done
echo done
