#!/bin/bash
# bench ms/step with device-memory kernel arguments forced on / off (HIP_FORCE_DEV_KERNARG)
for v in 1 0 1 0; do
  HIP_FORCE_DEV_KERNARG=$v timeout -k 10 120 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-host-staged --no-fp32-line > gpurun_out/ka_$v.json 2>/dev/null || { echo "kernarg $v failed"; continue; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/ka_$v.json').read().strip().splitlines()[-1]); print('DEV_KERNARG=$v', d['ms_per_step'], d['kernel_us'])"
done
