#!/bin/bash
# Round 5, call X: bf16 conv weight gradients on 2 groups -- parity subset, then bf16 variants.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05x
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_parity_full.py tests/test_gpu_dp.py tests/test_gpu_dp_c3.py tests/test_gpu_ppo.py -x -q --timeout 300 --timeout-method thread -m gpu > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
BENCH_ARGS="--dtype bf16" bash tools/r05_ab.sh r05x/ab bg2_g1 bg2_s384 bg2_s192
