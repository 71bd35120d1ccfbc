#!/bin/bash
# frames per workgroup of the per-frame conv kernels (forward conv12, backward conv12)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/fpw
mkdir -p $O
for cfg in "0 5" "6 5" "8 5" "0 6" "0 8" "6 6"; do
  set -- $cfg
  IMPALA_C12F_FPW=$1 IMPALA_C1_FPW=$2 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/f$1_b$2 -o run --output-format csv -- python3 bench.py --steps 100 --no-cpu-baseline --no-host-staged --roofline-kernel conv1_fwd_conv2_fwd > $O/bench_f$1_b$2.json 2> $O/f$1_b$2.err || exit $?
  IMPALA_C12F_FPW=$1 IMPALA_C1_FPW=$2 timeout -k 10 200 python bench.py --steps 200 --no-cpu-baseline --no-host-staged > $O/wall_f$1_b$2.json 2> $O/wall_f$1_b$2.err || exit $?
done
