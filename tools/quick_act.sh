#!/bin/bash
# learner / act GPU tests + smoke (gpurun_out/qa/)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/qa
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_learner.py tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit $?
