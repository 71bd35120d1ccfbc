#!/bin/bash
# Serial-stream kernel durations (no side-stream overlap): rocprofv3 --kernel-trace --stats.
set -o pipefail
OUT=gpurun_out/ser
rm -rf $OUT; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --roofline-kernel conv2_dgrad_conv1_wgrad "$@" > $OUT/b.json 2>$OUT/err
