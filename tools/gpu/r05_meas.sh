set -o pipefail
D=gpurun_out/r05_meas
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 240 python -u bench.py --no-cpu > $D/cfg3_views.json 2> $D/cfg3_views.err &&
timeout -k 10 240 python -u bench.py --no-cpu --layout packed > $D/cfg3_packed.json 2> $D/cfg3_packed.err &&
timeout -k 10 240 python -u bench.py --no-cpu --config 5 --replay 0 > $D/cfg5_r32.json 2> $D/cfg5_r32.err &&
timeout -k 10 240 python -u bench.py --no-cpu --config 5 --replay 0 --reserve 0 > $D/cfg5_r0.json 2> $D/cfg5_r0.err &&
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $D/ws5_r32 -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu --config 5 --replay 0 > $D/ws5_r32.log 2>&1 &&
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $D/ws5_r0 -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu --config 5 --replay 0 --reserve 0 > $D/ws5_r0.log 2>&1 &&
timeout -k 10 240 python -u tools/mirror_latency.py > $D/mirror_latency.json 2> $D/mirror_latency.err
