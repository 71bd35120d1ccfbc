#!/bin/bash
# Round 6 (gpurun_out/r06c/): rocprofv3 kernel trace of the drop-in loop over the device replay
# (tools/loop_trace.py), analysed per kernel: duration and the idle gap before each launch.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06c
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- python3 tools/loop_trace.py 300 > $O/loop.out 2> $O/loop.err || { echo "trace rc=$?"; tail -20 $O/loop.err; exit 1; }
python3 tools/loop_trace.py --analyse $O/trace 100 | tee $O/analysis.txt
