#!/bin/bash
# SAC GPU pass: parity tests, bf16 + fp32 bench, rocprofv3 kernel stats (gpurun_out/sac/)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/sac
timeout -k 10 300 python -u -m pytest tests/test_gpu_sac.py -x -q --timeout 120 --timeout-method thread > gpurun_out/sac/tests.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --algo sac --steps 200 --warmup 20 --cpu-seconds 12 > gpurun_out/sac/bench_bf16.json 2> gpurun_out/sac/bench_bf16.err || exit $?
timeout -k 10 200 python bench.py --algo sac --dtype fp32 --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/sac/bench_fp32.json 2> gpurun_out/sac/bench_fp32.err || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/sac/stats -o run --output-format csv -- python3 bench.py --algo sac --steps 50 --warmup 5 --no-cpu-baseline --roofline-kernel critic_fwd_chain > gpurun_out/sac/bench_stats.json 2> gpurun_out/sac/stats.err
echo "rocprof rc=$?"
