#!/bin/bash
# Round 6 (gpurun_out/r06u/): tools/loop_probe.py, the learner's host calls timed one by one.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06u
mkdir -p $O
for a in "host 2" "host 1" "device 2"; do
  timeout -k 10 200 python3 tools/loop_probe.py $a >> $O/probe.txt 2>&1 || { tail -20 $O/probe.txt; exit 1; }
done
cat $O/probe.txt | grep -v amdgpu.ids
