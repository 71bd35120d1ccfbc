#!/bin/bash
# Round 6 (gpurun_out/r06f/): the learner tests (prefetch), then the drop-in loop sub-record
# twice with the learner prefetching the next batch (ImpalaLearner prefetch=1, the default).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06f}
mkdir -p $O
fatal() { case $1 in 124|137|134|139) echo "fatal rc=$1 in $2"; exit 1;; esac; }
timeout -k 10 600 python -u -m pytest -v -s --timeout 120 --timeout-method thread tests/test_gpu_learner.py \
  > $O/learner_tests.log 2>&1; rc=$?; fatal $rc learner_tests
grep -E "PASSED|FAILED|Error" $O/learner_tests.log | tail -40
Q="--steps 20 --warmup 5 --no-alt-line --no-cpu-baseline"
for name in a b; do
  timeout -k 10 300 python bench.py $Q > $O/loop_$name.json 2> $O/loop_$name.err; rc=$?; fatal $rc loop_$name
  [ $rc = 0 ] || { echo "loop_$name rc=$rc"; tail -20 $O/loop_$name.err; continue; }
  python3 - $O/loop_$name.json $name <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
ll = d["learner_loop"]
print(sys.argv[2], "headline", d["ms_per_step"], "host_staged", d["host_staged"]["ms_per_step"])
for r in ("device_replay", "host_list_replay"):
    print("  ", r, {k: (v["ms_per_step"], v["ms_per_step_median"], v["host_ms_per_iter_median"]) for k, v in ll[r].items()})
PY
done
