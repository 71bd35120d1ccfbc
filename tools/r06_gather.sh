#!/bin/bash
# Round 6 (gpurun_out/$TAG/): the device-replay loop's kernel trace (tools/loop_trace.py: the
# gather's duration beside the step's kernels), then bench.py (the loop records).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06g}
mkdir -p $O
fatal() { case $1 in 124|137|134|139) echo "fatal rc=$1 in $2"; exit 1;; esac; }
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- python3 tools/loop_trace.py 300 > $O/loop.out 2> $O/loop.err; rc=$?; fatal $rc trace
[ $rc = 0 ] || { echo "trace rc=$rc"; tail -20 $O/loop.err; exit 1; }
python3 tools/loop_trace.py --analyse $O/trace 100 | tee $O/loop_analysis.txt
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err; rc=$?; fatal $rc bench
[ $rc = 0 ] || { echo "bench rc=$rc"; tail -30 $O/bench.err; exit 1; }
python3 - $O/bench.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print("headline", d["value"], d["ms_per_step"], "bf16", d["bf16_mode"]["ms_per_step"], "hs", d["host_staged"]["ms_per_step"])
ll = d["learner_loop"]
for r in ("device_replay", "host_list_replay"):
    print("  ", r, {k: (v["ms_per_step"], v["ms_per_step_median"]) for k, v in ll[r].items() if isinstance(v, dict)})
PY
