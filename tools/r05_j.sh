#!/bin/bash
# Round 5, call J: stamps of the pipelined LN body (lnp_st), then A/B with static priority.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05j
mkdir -p $O
IMPALA_HIP_LIB=build_variants/lnp_st.so timeout -k 10 120 python bench.py --steps 5 --warmup 2 --settle-ms 0 --no-cpu-baseline --no-host-staged --no-alt-line > $O/st.json 2> $O/st.err || { echo "stamps failed"; tail $O/st.err; exit 1; }
grep LNP $O/st.json | tail -14
bash tools/r05_ab.sh r05j/ab ln_old lnp_prio1 lnp_prio0
