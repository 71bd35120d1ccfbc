#!/bin/bash
# Round 5, call V: the weight-gradient bias sums split across the column tiles -- parity subset,
# then A/B fp32 and bf16 against the previous build.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05v
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity_full.py tests/test_gpu_parity.py tests/test_gpu_dp.py tests/test_gpu_ppo.py -x -q --timeout 300 --timeout-method thread -m gpu > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash tools/r05_ab.sh r05v/fp32 bias_base && BENCH_ARGS="--dtype bf16" bash tools/r05_ab.sh r05v/bf16 bias_base
