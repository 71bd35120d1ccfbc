#!/bin/bash
# fp32 forward: conv2 k-steps split over the two wave halves (conv1.h KSPL): the parity files,
# then bench A/B against build_variants/pre_c2k.so.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r05c2k}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_parity_full.py -x -q -m gpu --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash tools/r05_ab.sh ${1:-r05c2k}/ab pre_c2k || exit 1
