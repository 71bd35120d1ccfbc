#!/bin/bash
# Round 4: host-staged copy paths, third pass -- the new default (obs over 2 SDMA streams, small
# fields in one pull launch) against its neighbours, beside the fp32 step (tools/h2d_bw.py); the
# staging tests; bench.py's host_staged record; a rocprofv3 kernel trace of that pass.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r04hs3}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_learner.py tests/test_gpu_ppo.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/staging_tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/staging_tests.log; exit 1; }
tail -1 $O/staging_tests.log
run() {
  env "$@" timeout -k 10 120 python tools/h2d_bw.py 60 >> $O/h2d_bw.txt 2>&1 || { echo "h2d_bw $* rc=$?"; tail -5 $O/h2d_bw.txt; exit 1; }
  echo "  ^ $*" >> $O/h2d_bw.txt
}
run IMPALA_H2D_TAG=default
run IMPALA_H2D_SMALL_PULL=0
run IMPALA_H2D_STREAMS=1
run IMPALA_H2D_STREAMS=3
run IMPALA_H2D_STREAMS=4
run IMPALA_H2D_STREAMS=2 IMPALA_H2D_SMALL_PULL=0
run IMPALA_H2D_TAG=default_again
grep -A1 "H2D path" $O/h2d_bw.txt
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-alt-line --no-dp-variants > $O/bench.json 2> $O/bench.err || { echo "bench rc=$?"; tail -5 $O/bench.err; exit 1; }
python -c "import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print(d['value'], d.get('host_staged'))"
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/trace -o run -- python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-alt-line --no-dp-variants > $O/bench_trace.json 2> $O/trace.err || { echo "trace rc=$?"; tail -5 $O/trace.err; exit 1; }
ls -R $O/trace | head -20
python tools/hs_timeline.py $O/trace 6 | tee $O/timeline.txt
