#!/bin/bash
# IMPALA parity tests + bench + rocprof stats (gpurun_out/qi/)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/qi
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dp.py tests/test_gpu_learner.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --no-cpu-baseline --no-host-staged > $O/bench.json 2> $O/bench.err || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/stats -o run --output-format csv -- python3 bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-host-staged --roofline-kernel conv1_fwd_conv2_fwd > $O/bench_stats.json 2> $O/stats.err || exit $?
