#!/bin/bash
# round 3 probe: the parity tests whose printed numbers DESIGN quotes (-s), then smoke, bench
# and the rocprofv3 summaries (tools/profile.sh <tag>)
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-r03probe}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 400 python -u -m pytest -s -v --timeout 300 --timeout-method thread tests/test_gpu_parity_full.py "tests/test_gpu_parity.py::test_bf16_tracks_fp32_over_100_steps_c2" > $O/parity.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || exit $?
bash tools/profile.sh $TAG
