set -o pipefail
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/r06_base; mkdir -p $O
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 python -u bench.py --steps 20 --warmup 10 --no-cpu --no-packed > $O/bench_cfg3.json 2> $O/bench_cfg3.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --steps 20 --warmup 10 --no-cpu --no-packed > $O/bench_cfg3_prof.json 2> $O/prof.err &&
timeout -k 10 300 python -u bench.py --config 2 --steps 20 --warmup 10 --no-cpu --no-packed > $O/bench_cfg2.json 2> $O/bench_cfg2.err
