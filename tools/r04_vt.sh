#!/bin/bash
# Round 4: V-trace order + gradient modes on the GPU: the parity files verbose (printed
# figures), then the whole -m gpu suite, smoke(), the default bench line.  Each step under its
# own time limit; stop at the first failure.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r04a}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity_full.py tests/test_gpu_parity.py -v -s -m gpu --timeout 300 --timeout-method thread > $O/parity.log 2>&1 || { echo "parity rc=$?"; grep -E "FAIL|Error|assert" $O/parity.log | head -40; tail -5 $O/parity.log; exit 1; }
tail -2 $O/parity.log
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -30 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py ${BENCH_ARGS:-} > $O/bench.json 2> $O/bench.err || { echo "bench rc=$?"; tail -30 $O/bench.err; exit 1; }
cut -c1-400 $O/bench.json
