#!/bin/bash
# staging-ring parity (both copy modes), then the host-staged rate per pull-kernel grid size
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/stage
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_learner.py -x -q -k staging --timeout 120 --timeout-method thread > $O/test_staging.log 2>&1 || exit $?
for wg in 16 32 64 128; do
  IMPALA_H2D_KERNEL=$wg timeout -k 10 200 python bench.py --steps 50 --warmup 5 --no-cpu-baseline > $O/staged_pull$wg.json 2> $O/staged_pull$wg.err || exit $?
done
