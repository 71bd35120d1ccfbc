#!/bin/bash
# rocprofv3 kernel trace of bench.py's data-parallel step at world size 1 (RCCL group of one:
# the bucketed all-reduce path the N-GPU run takes), gpurun_out/dist1_prof/
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/dist1_prof
mkdir -p $O
export IMPALA_BENCH_DIST=1 RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29541
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/stats -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-fp32-line --no-host-staged "$@" > $O/bench.json 2> $O/bench.err || exit $?
echo done
