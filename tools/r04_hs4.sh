#!/bin/bash
# Round 4: host-staged loop shapes (tools/hs_loop.py) for the SDMA default on 1 / 2 streams, the
# all-SDMA variant and the round-3 pull kernel; then a kernel + memory-copy trace of the default.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r04hs4}
mkdir -p $O
run() {
  env "$@" timeout -k 10 150 python tools/hs_loop.py 200 >> $O/hs_loop.txt 2>&1 || { echo "hs_loop $* rc=$?"; tail -5 $O/hs_loop.txt; exit 1; }
}
run IMPALA_H2D_TAG=default
run IMPALA_H2D_STREAMS=1
run IMPALA_H2D_SMALL_PULL=0
run IMPALA_H2D_KERNEL=8
grep loop $O/hs_loop.txt
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/trace -o run -- python3 tools/hs_loop.py 40 > $O/trace_loop.txt 2> $O/trace.err || { echo "trace rc=$?"; tail -5 $O/trace.err; exit 1; }
cat $O/trace_loop.txt | grep loop
