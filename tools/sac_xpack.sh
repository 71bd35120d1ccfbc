#!/bin/bash
# SAC chain kernels with and without XCD packing: parity tests with packing, bench + rocprof both ways
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/xp
mkdir -p $O
SAC_XCD_PACK=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_sac.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit $?
for x in 0 1; do
  SAC_XCD_PACK=$x timeout -k 10 200 python bench.py --algo sac --steps 300 --warmup 20 --no-cpu-baseline > $O/bench$x.json 2> $O/bench$x.err || exit $?
  SAC_XCD_PACK=$x timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/s$x -o run --output-format csv -- python3 bench.py --algo sac --steps 50 --warmup 5 --no-cpu-baseline --roofline-kernel actor_chain > $O/bs$x.json 2> $O/s$x.err || exit $?
done
