#!/bin/bash
# PP stamp lines + bench ms of each build_variants/*.so with the split (non-fused) backward launch
for so in build_variants/*.so; do
  n=$(basename $so .so)
  IMPALA_LC12=${LC12:-0} IMPALA_HIP_LIB=$so timeout -k 10 120 python bench.py --steps 30 --warmup 3 --no-cpu-baseline --no-host-staged --no-fp32-line > gpurun_out/st_$n.log 2>&1 || { echo "variant $n: exit $?"; exit 1; }
  echo "== $n $(grep '^{' gpurun_out/st_$n.log | python -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["ms_per_step"], d["kernel_us"].get("conv2_dgrad_conv1_wgrad"))')"
  grep -E '^(PP|LN) ' gpurun_out/st_$n.log | tail -2
done
