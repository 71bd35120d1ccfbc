#!/bin/bash
# The driver's round-end GPU commands on this tree (gpurun_out/driver/): pytest -m gpu -x -q,
# smoke(), then the default bench line (N=1).  Each step under its own time limit.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/driver
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -30 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py ${BENCH_ARGS:-} > $O/bench.json 2> $O/bench.err || { echo "bench rc=$?"; tail -30 $O/bench.err; exit 1; }
cut -c1-600 $O/bench.json
