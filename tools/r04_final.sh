#!/bin/bash
# Round-4 rehearsal on the final tree: the whole -m gpu suite, smoke(), the default bench line
# (N=1: cpu baseline, host-staged, bf16 sub-record), then tools/profile.sh (rocprofv3 stats and
# the FETCH_SIZE / WRITE_SIZE passes) for the fp32 headline.  Stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
TAG=${TAG:-r04x}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/gpu_tests.log; exit 1; }
tail -3 $O/gpu_tests.log
IMPALA_HIP_LIB=$PWD/impala_amd/libimpala_hip_ab.so timeout -k 10 600 python -u -m pytest tests/test_gpu_ab_variants.py -x -q -m gpu --timeout 300 --timeout-method thread > $O/gpu_ab_tests.log 2>&1 || { echo "ab tests rc=$?"; tail -30 $O/gpu_ab_tests.log; exit 1; }
tail -1 $O/gpu_ab_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -30 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { echo "bench rc=$?"; tail -10 $O/bench.err; exit 1; }
tail -c 600 $O/bench.json
timeout -k 10 1000 bash tools/profile.sh $TAG > $O/profile.log 2>&1 || { echo "profile rc=$?"; tail -10 $O/profile.log; exit 1; }
tail -2 $O/profile.log
