#!/bin/bash
# Kernel traces of the bf16 and fp32 steps with direct launches and with hipGraph replay
# (IMPALA_GRAPH=1): per-kernel durations and the idle gap before each launch
# (tools/kernel_gaps.py gpurun_out/<tag>).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r05gt}
mkdir -p $O
for dt in bf16 fp32; do
  for g in 0 1; do
    IMPALA_GRAPH=$g timeout -k 10 200 rocprofv3 --kernel-trace -d $O/$dt.g$g -o run --output-format csv -- python3 bench.py --steps 50 --warmup 10 --dtype $dt --no-cpu-baseline --no-host-staged --no-alt-line > $O/$dt.g$g.json 2> $O/$dt.g$g.err || { echo "$dt g$g rc=$?"; tail -5 $O/$dt.g$g.err; exit 1; }
  done
done
echo done
