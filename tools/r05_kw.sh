#!/bin/bash
# The FC forward's wave k-split (gemm_tile_body KW): parity files on the product, then bench A/B
# fp32 (product vs fckw_off) and bf16 (product vs fckw_bf16).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r05kw}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_parity_full.py -x -q -m gpu --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash tools/r05_ab.sh ${1:-r05kw}/ab ${VARS:-fckw_off} || exit 1
[ -n "$BF16_VARS" ] && { BENCH_ARGS="--dtype bf16" bash tools/r05_ab.sh ${1:-r05kw}/abb $BF16_VARS || exit 1; }; true
