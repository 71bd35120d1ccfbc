#!/bin/bash
# Round 6 (gpurun_out/r06k/): FC weight-gradient splits (IMPALA_FC_WG: target workgroups of the
# split plan; 64 -> 4 splits, 128 -> 8 (fp32 default), 256 -> 16) and the reduction's loads per
# thread (IMPALA_RED_LPT), fp32 and bf16, 200-step headline regions with the per-kernel table.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06k
mkdir -p $O
fatal() { case $1 in 124|137|134|139) echo "fatal rc=$1 in $2"; exit 1;; esac; }
Q="--steps 200 --warmup 20 --no-alt-line --no-cpu-baseline --no-host-staged --no-learner-loop"
for dt in fp32 bf16; do
for v in "base:" "fc64:IMPALA_FC_WG=64" "fc256:IMPALA_FC_WG=256" "lpt8:IMPALA_RED_LPT=8" "lpt32:IMPALA_RED_LPT=32" "base2:"; do
  name=${v%%:*}; envs=${v#*:}
  env $envs timeout -k 10 200 python bench.py $Q --dtype $dt > $O/${dt}_$name.json 2> $O/${dt}_$name.err; rc=$?; fatal $rc $name
  [ $rc = 0 ] || { echo "$dt $name rc=$rc"; tail -5 $O/${dt}_$name.err; continue; }
  python3 -c "import json;d=json.load(open('$O/${dt}_$name.json'));k=d['kernel_us'];print('$dt $name', d['ms_per_step'], d['ms_per_step_median'], 'fc_bwd', k.get('fc_wgrad_fc_dgrad'), 'red', k.get('reduce_grads'))"
done
done
