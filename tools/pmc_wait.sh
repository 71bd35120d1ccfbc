#!/bin/bash
# One rocprofv3 PMC pass over the fp32 bench: where the learner kernels' waves spend their cycles
# (MI355X_MICROARCH.md PMC slots: WAIT_ANY = parked on s_waitcnt / barrier, WAIT_INST_ANY =
# issue-stalled, ACTIVE_INST_ANY = issuing; the three are disjoint and sum to WAVE_CYCLES) and
# the instruction mix.  tools/pmc_util.py-style summary via tools/pmc_table.py <dir>.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05pmcw}
mkdir -p $O
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA --kernel-trace --output-format csv -d $O/pmc -o run -- python3 bench.py --steps 20 --warmup 20 --settle-ms 0 --no-cpu-baseline --no-host-staged --no-alt-line --no-dp-variants --no-learner-loop --no-actor-act ${BENCH_ARGS:-} > $O/bench.json 2> $O/pmc.err || { echo "pmc rc=$?"; tail -5 $O/pmc.err; exit 1; }
echo pmc done
