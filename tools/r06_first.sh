#!/bin/bash
# Round 6, first GPU pass (gpurun_out/r06a/): the new / changed GPU tests verbosely (C3 at
# world 8, the drop-in learner vs fp64, row staging), then the whole -m gpu suite, the driver's
# bench line, and the graph-replay A/B with the step clock off.  Each step under its own limit;
# a test failure is reported and the pass goes on, a time limit / abort / fault ends it.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06a
mkdir -p $O
fatal() { case $1 in 124|137|134|139) echo "fatal rc=$1 in $2"; exit 1;; esac; }
timeout -k 10 600 python -u -m pytest -v -s --timeout 500 --timeout-method thread \
  tests/test_gpu_learner.py tests/test_gpu_dp_c3.py -k "c3_replicas or builder_learner or pinned_replay or agent_train" \
  > $O/new_tests.log 2>&1; rc=$?; fatal $rc new_tests
grep -E "PASSED|FAILED|C3 |learner |Error" $O/new_tests.log | tail -40
timeout -k 10 900 python -u -m pytest tests -q -m gpu --timeout 500 --timeout-method thread > $O/tests.log 2>&1; rc=$?; fatal $rc tests
tail -5 $O/tests.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err; rc=$?; fatal $rc bench
[ $rc = 0 ] || { echo "bench rc=$rc"; tail -30 $O/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench.json'));print(d['value'],d['ms_per_step'],d['roofline']['avg_launch_us']);print(json.dumps(d['learner_loop'])[:3000])"
for g in 0 1; do
  IMPALA_GRAPH=$g timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-step-clock --no-alt-line --no-cpu-baseline --no-host-staged --no-learner-loop > $O/graph$g.json 2> $O/graph$g.err; rc=$?; fatal $rc graph$g
  python3 -c "import json;d=json.load(open('$O/graph$g.json'));print('graph$g', d['ms_per_step'])"
done
