#!/bin/bash
# Round 6 (gpurun_out/r06e/): the drop-in loop sub-record with the streaming-store row collate
# on 8 / 12 / 16 pool threads (IMPALA_STAGE_THREADS), host_staged beside it.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06e
mkdir -p $O
fatal() { case $1 in 124|137|134|139) echo "fatal rc=$1 in $2"; exit 1;; esac; }
Q="--steps 20 --warmup 5 --no-alt-line --no-cpu-baseline"
for v in "t8:IMPALA_STAGE_THREADS=8" "t12:IMPALA_STAGE_THREADS=12" "t16:IMPALA_STAGE_THREADS=16" "t8b:IMPALA_STAGE_THREADS=8"; do
  name=${v%%:*}; envs=${v#*:}
  env $envs timeout -k 10 300 python bench.py $Q > $O/loop_$name.json 2> $O/loop_$name.err; rc=$?; fatal $rc loop_$name
  [ $rc = 0 ] || { echo "loop_$name rc=$rc"; tail -20 $O/loop_$name.err; continue; }
  python3 - $O/loop_$name.json $name <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
ll = d["learner_loop"]
print(sys.argv[2], "headline", d["ms_per_step"], "host_staged", d["host_staged"]["ms_per_step"])
for r in ("device_replay", "pinned_replay", "host_list_replay"):
    print("  ", r, {k: (v["ms_per_step"], v["ms_per_step_median"], v["host_ms_per_iter_median"]) for k, v in ll[r].items()})
PY
done
