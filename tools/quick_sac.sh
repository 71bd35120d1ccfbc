#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/qs
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_sac.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --algo sac --steps 200 --warmup 20 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/stats -o run --output-format csv -- python3 bench.py --algo sac --steps 50 --warmup 5 --no-cpu-baseline --roofline-kernel actor_chain > $O/bench_stats.json 2> $O/stats.err || exit $?
