# the whole GPU suite, the scalar call with and without the zero-copy block, config 4's kernel order
# per step (rocprofv3, same process as its bench line), config 3 and 4 bench lines
set -o pipefail
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/r06_p; mkdir -p $O
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -u tools/mirror_latency.py > $O/mirror_zc.json 2> $O/mirror_zc.err || { tail -20 $O/mirror_zc.err; exit 1; }
IE_SMALL_ZC=0 timeout -k 10 300 python -u tools/mirror_latency.py > $O/mirror_nozc.json 2> $O/mirror_nozc.err || { tail -20 $O/mirror_nozc.err; exit 1; }
cut -c1-330 $O/mirror_zc.json; cut -c1-330 $O/mirror_nozc.json
timeout -k 10 300 python -u tools/task_times.py > $O/task_times.json 2> $O/task_times.err || { tail -20 $O/task_times.err; exit 1; }
cut -c1-300 $O/task_times.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof4 -o run -- python3 bench.py --config 4 --steps 20 --warmup 10 --no-cpu --replay 0 > $O/bench_cfg4_prof.json 2> $O/prof4.err || { tail -20 $O/prof4.err; exit 1; }
for c in 3 4; do
  timeout -k 10 300 python -u bench.py --config $c --no-cpu --no-packed > $O/bench_cfg$c.json 2> $O/bench_cfg$c.err || { tail -20 $O/bench_cfg$c.err; exit 1; }
  tail -1 $O/bench_cfg$c.json | cut -c1-200
done
