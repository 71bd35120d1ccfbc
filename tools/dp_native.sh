#!/bin/bash
# native RCCL data-parallel step at world size 1: the bitwise tests, then the bench's DP code
# path (torch.distributed.run, one rank) with the native communicator (1 and 2 buckets) and the
# c10d all-reduce, fp32 headline + bf16 sub-record
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/dp_native
mkdir -p $O
timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_gpu_dp_c3.py -k "native or rccl" > $O/tests.log 2>&1 || exit $?
for mode in "1 2" "1 1" "0 1"; do
  set -- $mode
  IMPALA_BENCH_DIST=1 IMPALA_DP_NATIVE=$1 IMPALA_DP_BUCKETS=$2 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr=127.0.0.1 --master-port=29533 bench.py --no-cpu-baseline --no-host-staged > $O/bench_native$1_b$2.json 2> $O/bench_native$1_b$2.err || exit $?
done
echo done
