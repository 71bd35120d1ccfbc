#!/bin/bash
# Round 6 (gpurun_out/r06b/): the learner-path GPU tests, then the drop-in loop sub-record
# (bench.py learner_loop) under the row-staging modes: host collate on 8 / 4 / 16 threads
# (IMPALA_STAGE_THREADS) and one SDMA copy per row (IMPALA_STAGE_ROWS=rows).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06b
mkdir -p $O
fatal() { case $1 in 124|137|134|139) echo "fatal rc=$1 in $2"; exit 1;; esac; }
timeout -k 10 600 python -u -m pytest -v -s --timeout 300 --timeout-method thread tests/test_gpu_learner.py \
  > $O/learner_tests.log 2>&1; rc=$?; fatal $rc learner_tests
grep -E "PASSED|FAILED|learner |Error" $O/learner_tests.log | tail -40
Q="--steps 20 --warmup 5 --no-alt-line --no-cpu-baseline --no-host-staged"
for v in "default:" "t4:IMPALA_STAGE_THREADS=4" "t16:IMPALA_STAGE_THREADS=16" "rows:IMPALA_STAGE_ROWS=rows"; do
  name=${v%%:*}; envs=${v#*:}
  env $envs timeout -k 10 300 python bench.py $Q > $O/loop_$name.json 2> $O/loop_$name.err; rc=$?; fatal $rc loop_$name
  [ $rc = 0 ] || { echo "loop_$name rc=$rc"; tail -20 $O/loop_$name.err; continue; }
  python3 - $O/loop_$name.json $name <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
ll = d["learner_loop"]
print(sys.argv[2], "headline", d["ms_per_step"])
for r in ("device_replay", "pinned_replay", "host_list_replay"):
    print("  ", r, {k: (v["ms_per_step"], v["ms_per_step_median"], v["host_ms_per_iter_median"]) for k, v in ll[r].items()})
PY
done
