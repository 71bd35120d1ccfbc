#!/bin/bash
# Serial-stream kernel durations of each build_variants/*.so (tools/variants.py) on the GPU box.
set -o pipefail
export TMPDIR=/tmp
for so in build_variants/*.so; do
  n=$(basename $so .so)
  OUT=gpurun_out/var_$n
  rm -rf $OUT; mkdir -p $OUT
  IMPALA_HIP_LIB=$so timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --roofline-kernel conv2_dgrad_conv1_wgrad > $OUT/b.json 2>$OUT/err || echo "variant $n: bench exit $?"
done
