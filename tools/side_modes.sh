#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/side
mkdir -p $O
IMPALA_SIDE_STREAM=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dp.py -x -q --timeout 120 --timeout-method thread > $O/tests2.log 2>&1 || exit $?
for m in 0 1 2 3; do
  IMPALA_SIDE_STREAM=$m timeout -k 10 200 python bench.py --steps 300 --no-cpu-baseline --no-host-staged > $O/b$m.json 2> $O/b$m.err || exit $?
done
for m in 0 2; do
  IMPALA_SIDE_STREAM=$m timeout -k 10 200 python bench.py --steps 300 --no-cpu-baseline --no-host-staged > $O/c$m.json 2> $O/c$m.err || exit $?
done
