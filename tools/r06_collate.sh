#!/bin/bash
# Round 6 (gpurun_out/r06s/): tools/collate_probe.py on 1 / 4 / 8 / 16 staging pool threads.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06s
mkdir -p $O
for t in 8 16 4; do
  IMPALA_STAGE_THREADS=$t timeout -k 10 120 python3 tools/collate_probe.py 2>&1 | tee -a $O/probe.txt | grep threads || exit 1
done
