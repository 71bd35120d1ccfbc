#!/bin/bash
# Round 6 (gpurun_out/r06l/): the library built with other LLVM scheduling strategies
# (tools/build_flag_variants.py -> build_variants/) against the default build, 200-step
# headline regions, fp32 and bf16, interleaved.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06l
mkdir -p $O
fatal() { case $1 in 124|137|134|139) echo "fatal rc=$1 in $2"; exit 1;; esac; }
Q="--steps 200 --warmup 20 --no-alt-line --no-cpu-baseline --no-host-staged --no-learner-loop"
for dt in fp32 bf16; do
for v in default maxilp memclause trackers bias0 default2; do
  lib=impala_amd/libimpala_hip.so
  case $v in default*) ;; *) lib=build_variants/libimpala_hip_$v.so;; esac
  IMPALA_HIP_LIB=$PWD/$lib timeout -k 10 200 python bench.py $Q --dtype $dt > $O/${dt}_$v.json 2> $O/${dt}_$v.err; rc=$?; fatal $rc $v
  [ $rc = 0 ] || { echo "$dt $v rc=$rc"; tail -5 $O/${dt}_$v.err; continue; }
  python3 -c "import json;d=json.load(open('$O/${dt}_$v.json'));k=d['kernel_us'];print('$dt $v', d['ms_per_step'], d['ms_per_step_median'], {a[:14]: b for a, b in k.items()})"
done
done
