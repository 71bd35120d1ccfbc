#!/bin/bash
# Round 6 rehearsal on the final tree (gpurun_out/${TAG}/): the whole -m gpu suite (verbose),
# the BASELINE-size parity file with its printed margins (-s), smoke(), the driver's bench
# command twice, then rocprofv3 kernel stats + HBM bytes for fp32 and bf16 (tools/profile.sh).
# A test failure is reported and the pass goes on; a time limit / abort / fault ends it.
set -o pipefail
export TMPDIR=/tmp
TAG=${TAG:-r06final}
O=gpurun_out/$TAG
mkdir -p $O
fatal() { case $1 in 124|137|134|139) echo "fatal rc=$1 in $2"; exit 1;; esac; }
timeout -k 10 900 python -u -m pytest tests -v -m gpu --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?; fatal $rc tests
tail -3 $O/tests.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity_full.py -v -s --timeout 120 --timeout-method thread > $O/parity.log 2>&1; rc=$?; fatal $rc parity
tail -2 $O/parity.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?; fatal $rc smoke
tail -1 $O/smoke.log
for i in 1 2; do
  timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench$i.json 2> $O/bench$i.err; rc=$?; fatal $rc bench$i
  python3 -c "import json;d=json.load(open('$O/bench$i.json'));print('bench$i', d['value'], d['ms_per_step'], d['ms_per_step_median'], 'bf16', d['bf16_mode']['ms_per_step'], 'hs', d['host_staged']['ms_per_step'], 'loop', d['learner_loop']['device_replay']['sync_every_100']['ms_per_step'], d['learner_loop']['host_list_replay']['sync_every_100']['ms_per_step'])"
done
bash tools/profile.sh ${TAG}p || exit 1
bash tools/profile.sh ${TAG}pb --dtype bf16 || exit 1
