#!/bin/bash
# Round 6 (gpurun_out/r06v/): bench.py's learner_loop record alone in a fresh process, beside
# the direct learner loop (tools/loop_probe.py).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06v
mkdir -p $O
for a in "bench" "host 2" "bench"; do
  timeout -k 10 200 python3 tools/loop_probe.py $a >> $O/probe.txt 2>&1 || { tail -20 $O/probe.txt; exit 1; }
done
grep -E "bench-loop|per train_step" $O/probe.txt
