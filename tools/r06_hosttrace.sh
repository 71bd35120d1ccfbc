#!/bin/bash
# Round 6 (gpurun_out/r06t/): kernel + memory-copy trace of the drop-in loop over the host
# replay (tools/loop_trace.py ... host), analysed per step.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06t
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/trace -o run -- python3 tools/loop_trace.py 300 host > $O/loop.out 2> $O/loop.err || { echo "trace rc=$?"; tail -20 $O/loop.err; exit 1; }
python3 tools/loop_trace.py --analyse $O/trace 100 | tee $O/analysis.txt
head -3 $(ls $O/trace/*memory_copy_trace.csv | head -1) 2>/dev/null || find $O/trace -name "*copy*" | head
