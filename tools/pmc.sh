#!/bin/bash
# SQ/LDS counter passes over a short bench run (one --pmc group per rocprofv3 run, each group
# within the per-pass hardware limits: <= 8 SQ_, <= 2 GRBM_), plus the kernel trace's register /
# LDS / workgroup-size columns.  usage: tools/pmc.sh <tag> [bench args...]
set -o pipefail
TAG=${1:-pmc}; shift
OUT=gpurun_out/pmc_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
ARGS="--steps 10 --warmup 2 --no-cpu-baseline --no-fp32-line --no-host-staged --no-learner-loop --no-actor-act $@"
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VMEM GRBM_GUI_ACTIVE" ; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace -d $OUT/p$i -o run --output-format csv -- python3 bench.py $ARGS > $OUT/bench$i.json 2> $OUT/p$i.err || { echo "pass $i failed"; tail -5 $OUT/p$i.err; exit 1; }
done
echo pmc done
