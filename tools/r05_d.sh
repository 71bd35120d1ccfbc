#!/bin/bash
# Round 5, call D: which runtime call holds the host-staged stall -- HIP + HSA API traces of
# tools/hs_calls.py (the pinned-buffer hypothesis: a hipMemcpyAsync source not recognised as
# page-locked is locked on the fly), plus the pull-kernel copy path for comparison.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05d
mkdir -p $O
IMPALA_H2D_KERNEL=8 timeout -k 10 200 python3 tools/hs_calls.py 5 20 > $O/hs_pull.txt 2>&1 || { echo "pull rc=$?"; tail $O/hs_pull.txt; exit 1; }
cd /tmp
timeout -k 10 300 rocprofv3 --hip-runtime-trace --hsa-trace --memory-copy-trace --kernel-trace -d $GRAFT_REPO_ROOT/$O/api -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/hs_calls.py 5 20 > $GRAFT_REPO_ROOT/$O/hs_api.txt 2>&1 || { echo "trace rc=$?"; tail $GRAFT_REPO_ROOT/$O/hs_api.txt; exit 1; }
echo done
