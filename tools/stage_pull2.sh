#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/stage2
mkdir -p $O
for wg in 4 8 12 16; do
  IMPALA_H2D_KERNEL=$wg timeout -k 10 200 python bench.py --steps 50 --warmup 5 --no-cpu-baseline > $O/staged_pull$wg.json 2> $O/staged_pull$wg.err || exit $?
done
