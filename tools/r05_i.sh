#!/bin/bash
# Round 5, call I: the pipelined fp32 LayerNorm / conv3-dgrad body -- parity tests, then A/B.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05i
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity_full.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -m gpu > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash tools/r05_ab.sh r05i/ab ln_old
