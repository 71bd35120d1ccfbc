#!/bin/bash
# Round 6 (gpurun_out/$TAG/): the replay ring read in place by the learner step
# (impala_train_step_rows) -- the learner and parity GPU tests, then the loop records
# (tools/loop_probe.py bench) with the rows path (default) and with gathers
# (IMPALA_REPLAY_ROWS=0), twice each, then the driver's bench command.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06rows}
mkdir -p $O
fatal() { case $1 in 124|137|134|139) echo "fatal rc=$1 in $2"; exit 1;; esac; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_learner.py tests/test_gpu_parity.py -v -m gpu --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?; fatal $rc tests
tail -2 $O/tests.log
[ $rc = 0 ] || { grep -E "FAIL|Error" $O/tests.log | head -20; exit 1; }
for r in a b; do
  for g in 1 0; do
    IMPALA_REPLAY_ROWS=$g timeout -k 10 300 python tools/loop_probe.py bench > $O/loop_${g}_$r.txt 2>&1; rc=$?; fatal $rc loop
    echo "rows=$g $r $(grep bench-loop $O/loop_${g}_$r.txt | head -1)"
    IMPALA_REPLAY_ROWS=$g timeout -k 10 200 python tools/sync1_probe.py 300 > $O/probe_${g}_$r.txt 2>&1; rc=$?; fatal $rc probe
    echo "rows=$g $r $(grep 'ms per step' $O/probe_${g}_$r.txt) / read->call $(grep 'read -> next' $O/probe_${g}_$r.txt | awk '{print $6}')"
  done
done
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err; rc=$?; fatal $rc bench
python3 - $O/bench.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print("headline", d["value"], d["ms_per_step"], "bf16", d["bf16_mode"]["ms_per_step"], "hs", d["host_staged"]["ms_per_step"])
ll = d["learner_loop"]
for r in ("device_replay", "host_list_replay"):
    print("  ", r, {k: (v["ms_per_step"], v["ms_per_step_median"]) for k, v in ll[r].items() if isinstance(v, dict)})
PY
