#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/qr
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dp.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --no-cpu-baseline --no-host-staged > $O/bench.json 2> $O/bench.err || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/stats -o run --output-format csv -- python3 bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-host-staged --roofline-kernel reduce_grads > $O/bench_stats.json 2> $O/stats.err || exit $?
