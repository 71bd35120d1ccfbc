#!/bin/bash
# round-end rehearsal (gpurun_out/rehearse/): the whole -m gpu suite, smoke(), the default bench
# line, then rocprofv3 kernel stats + PMC HBM bytes of the bench (tools/profile.sh <tag>)
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-rehearse}
O=gpurun_out/rehearse
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || exit $?
bash tools/profile.sh $TAG
