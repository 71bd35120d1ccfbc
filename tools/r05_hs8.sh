#!/bin/bash
# head_step on 8 column slices per trajectory group (head.h head_split, fp32): parity files (+ PPO),
# bench A/B fp32 and bf16 against build_variants/pre_hs8.so.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r05hs8}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_parity_full.py tests/test_gpu_ppo.py -x -q -m gpu --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash tools/r05_ab.sh ${1:-r05hs8}/ab pre_hs8 || exit 1
BENCH_ARGS="--dtype bf16" bash tools/r05_ab.sh ${1:-r05hs8}/abb pre_hs8 || exit 1
