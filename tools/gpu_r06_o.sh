set -o pipefail
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/r06_o; mkdir -p $O
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -u tools/mirror_latency.py > $O/mirror_latency.json 2> $O/mirror.err || { tail -20 $O/mirror.err; exit 1; }
cat $O/mirror_latency.json | cut -c1-400
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof4 -o run -- python3 bench.py --config 4 --steps 20 --warmup 10 --no-cpu --replay 0 > $O/bench_cfg4_prof.json 2> $O/prof4.err || { tail -20 $O/prof4.err; exit 1; }
tail -1 $O/bench_cfg4_prof.json | cut -c1-300
