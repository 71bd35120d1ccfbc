#!/bin/bash
# SQ/LDS counter passes over a short bench run (one --pmc group per rocprofv3 run).
set -o pipefail
TAG=${1:-pmc}; shift
OUT=gpurun_out/pmc_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
ARGS="--steps 10 --warmup 2 --no-cpu-baseline --roofline-kernel conv2_dgrad_conv1_wgrad $@"
rocprofv3 -L > $OUT/counters.txt 2>&1 || true
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE" ; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace -d $OUT/p$i -o run --output-format csv -- python3 bench.py $ARGS > $OUT/bench$i.json 2> $OUT/p$i.err || { echo "pass $i failed"; tail -5 $OUT/p$i.err; }
done
echo pmc done
