#!/bin/bash
# Round 5, call N: weight-gradient Y-row cursors -- parity subset (bitwise launch modes, full
# step vs fp64), then A/B fp32 and bf16 against the HEAD build.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05n
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity_full.py tests/test_gpu_parity.py tests/test_gpu_dp.py -x -q --timeout 300 --timeout-method thread -m gpu > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash tools/r05_ab.sh r05n/fp32 wg_base && BENCH_ARGS="--dtype bf16" bash tools/r05_ab.sh r05n/bf16 wg_base
