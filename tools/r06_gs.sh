#!/bin/bash
# Round 6 (gpurun_out/$TAG/): the device replay's gather on its own stream (IMPALA_GATHER_STREAM)
# -- the learner GPU tests, then the loop records (tools/loop_probe.py bench) and the sync-1
# probe with the gather on the learner's stream (0) and on its own (1), twice each.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06gs}
mkdir -p $O
fatal() { case $1 in 124|137|134|139) echo "fatal rc=$1 in $2"; exit 1;; esac; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_learner.py -v -m gpu --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?; fatal $rc tests
tail -2 $O/tests.log
[ $rc = 0 ] || { grep -E "FAIL|Error" $O/tests.log | head; exit 1; }
for r in a b; do
  for g in 0 1; do
    IMPALA_GATHER_STREAM=$g timeout -k 10 300 python tools/loop_probe.py bench > $O/loop_${g}_$r.txt 2>&1; rc=$?; fatal $rc loop
    echo "gs=$g $r $(grep bench-loop $O/loop_${g}_$r.txt | head -1)"
    IMPALA_GATHER_STREAM=$g timeout -k 10 200 python tools/sync1_probe.py 300 > $O/probe_${g}_$r.txt 2>&1; rc=$?; fatal $rc probe
    echo "gs=$g $r $(grep 'ms per step' $O/probe_${g}_$r.txt)"
  done
done
