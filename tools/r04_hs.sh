#!/bin/bash
# Round 4: the host-staged path -- H2D ring rate alone and beside the fp32 step for the pull
# kernel at 8 / 16 / 32 workgroups and for hipMemcpyAsync (SDMA), then a rocprofv3 kernel trace
# of bench.py's host_staged pass (tools/hs_timeline.py reads it).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r04hs}
mkdir -p $O
for wg in 8 16 32 0; do
  IMPALA_H2D_KERNEL=$wg timeout -k 10 120 python tools/h2d_bw.py 40 >> $O/h2d_bw.txt 2>&1 || { echo "h2d_bw $wg rc=$?"; tail -5 $O/h2d_bw.txt; exit 1; }
done
cat $O/h2d_bw.txt | grep "H2D path"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-alt-line > $O/bench_trace.json 2> $O/trace.err || { echo "trace rc=$?"; tail -5 $O/trace.err; exit 1; }
python tools/hs_timeline.py $O/trace 6
