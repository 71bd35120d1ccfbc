#!/bin/bash
# Round 5, call B: per-step marker A/B (tools/marker_ab.py, plain and under a kernel trace) and
# the host-staged stall's location (tools/hs_calls.py in fresh processes, per copy path).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05b
mkdir -p $O
timeout -k 10 200 python3 tools/marker_ab.py 100 fp32 > $O/marker_fp32.txt 2>&1 || { echo "marker rc=$?"; tail $O/marker_fp32.txt; exit 1; }
timeout -k 10 200 python3 tools/marker_ab.py 100 bf16 > $O/marker_bf16.txt 2>&1 || { echo "marker bf16 rc=$?"; tail $O/marker_bf16.txt; exit 1; }
timeout -k 10 200 python3 tools/hs_calls.py 5 20 > $O/hs_default.txt 2>&1 || { echo "hs rc=$?"; tail $O/hs_default.txt; exit 1; }
IMPALA_H2D_STREAMS=1 timeout -k 10 200 python3 tools/hs_calls.py 5 20 > $O/hs_1stream.txt 2>&1 || { echo "hs1 rc=$?"; exit 1; }
IMPALA_H2D_SMALL_PULL=0 timeout -k 10 200 python3 tools/hs_calls.py 5 20 > $O/hs_nopull.txt 2>&1 || { echo "hs2 rc=$?"; exit 1; }
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $GRAFT_REPO_ROOT/$O/trace_marker -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/marker_ab.py 100 fp32 > $GRAFT_REPO_ROOT/$O/marker_trace.txt 2>&1 || { echo "trace rc=$?"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $GRAFT_REPO_ROOT/$O/trace_hs -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/hs_calls.py 5 20 > $GRAFT_REPO_ROOT/$O/hs_trace.txt 2>&1 || { echo "trace2 rc=$?"; exit 1; }
echo done
