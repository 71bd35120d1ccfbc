#!/bin/bash
# Round 6 (gpurun_out/$TAG/): shared copy streams + lazy capture stream — the learner tests, then
# the bench twice (host_staged now runs after the drop-in loop in the same process).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06x}
mkdir -p $O
fatal() { case $1 in 124|137|134|139) echo "fatal rc=$1 in $2"; exit 1;; esac; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_learner.py tests/test_gpu_parity.py -v -m gpu --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?; fatal $rc tests
tail -4 $O/tests.log
for i in 1 2; do
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench$i.json 2> $O/bench$i.err; rc=$?; fatal $rc bench
[ $rc = 0 ] || { echo "bench rc=$rc"; tail -30 $O/bench$i.err; exit 1; }
python3 - $O/bench$i.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print("headline", d["value"], d["ms_per_step"], "bf16", d["bf16_mode"]["ms_per_step"], "hs", d["host_staged"]["ms_per_step"])
ll = d["learner_loop"]
for r in ("device_replay", "host_list_replay"):
    print("  ", r, {k: (v["ms_per_step"], v["ms_per_step_median"]) for k, v in ll[r].items() if isinstance(v, dict)})
PY
done
