#!/bin/bash
# rocprofv3 kernel stats + HBM traffic counters for bench.py (run on the GPU box via gpurun).
# usage: tools/profile.sh <tag> [bench args...]
set -o pipefail
TAG=${1:-r01}; shift
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
ARGS="--steps 20 --warmup 20 --settle-ms 0 --no-cpu-baseline --no-fp32-line --no-host-staged --no-learner-loop --no-actor-act $@"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/stats -o run --output-format csv -- python3 bench.py $ARGS > $OUT/bench_stats.json 2> $OUT/stats.err || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $OUT/fetch -o run --output-format csv -- python3 bench.py $ARGS > $OUT/bench_fetch.json 2> $OUT/fetch.err || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $OUT/write -o run --output-format csv -- python3 bench.py $ARGS > $OUT/bench_write.json 2> $OUT/write.err || exit $?
echo profile done
