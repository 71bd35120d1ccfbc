#!/bin/bash
# reduce_grads split-group rule: loads per thread 2 / 4 / 8 / 16 (rocprof serial durations)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/red
mkdir -p $O
for l in 2 4 8 16; do
  IMPALA_RED_LPT=$l timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/l$l -o run --output-format csv -- python3 bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-host-staged --roofline-kernel reduce_grads > $O/bench$l.json 2> $O/l$l.err || exit $?
done
