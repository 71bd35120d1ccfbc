#!/bin/bash
# L1/L2 request counters for the SAC chains (per-CU weight streaming)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/sacpmc
mkdir -p $O
rocprofv3 -L > $O/counters.txt 2>&1 || true
timeout -s KILL 90 rocprofv3 --pmc TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCC_HIT_sum TCC_MISS_sum --kernel-trace -d $O/p1 -o run --output-format csv -- python3 bench.py --algo sac --steps 10 --warmup 2 --no-cpu-baseline --roofline-kernel actor_chain > $O/b1.json 2> $O/p1.err
echo "pmc rc=$?"
