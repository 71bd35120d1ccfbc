#!/bin/bash
# Round-end style GPU pass (gpurun_out/round/): the whole -m gpu suite, the default bench (IMPALA
# bf16, with the host-staged pass), the SAC bench, and rocprofv3 kernel stats of both benches.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/round
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit $?
timeout -k 10 300 python bench.py > $O/bench_impala_bf16.json 2> $O/bench_impala_bf16.err || exit $?
timeout -k 10 200 python bench.py --algo sac --steps 200 --warmup 20 --cpu-seconds 12 > $O/bench_sac_bf16.json 2> $O/bench_sac_bf16.err || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/stats_sac -o run --output-format csv -- python3 bench.py --algo sac --steps 50 --warmup 5 --no-cpu-baseline --roofline-kernel actor_chain > $O/bench_sac_stats.json 2> $O/stats_sac.err || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/stats_impala -o run --output-format csv -- python3 bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-host-staged --roofline-kernel conv1_fwd_conv2_fwd > $O/bench_impala_stats.json 2> $O/stats_impala.err
echo "rocprof rc=$?"
