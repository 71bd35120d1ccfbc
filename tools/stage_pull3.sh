#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/stage3
mkdir -p $O
for cfg in "8 256" "8 512" "8 1024" "16 512" "24 256" "32 1024"; do
  set -- $cfg
  IMPALA_H2D_KERNEL=$1 IMPALA_H2D_THREADS=$2 timeout -k 10 200 python bench.py --steps 50 --warmup 5 --no-cpu-baseline > $O/pull_$1_$2.json 2> $O/pull_$1_$2.err || exit $?
done
