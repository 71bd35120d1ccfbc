#!/bin/bash
# bench line (ms, per-kernel us) of each build_variants/*.so, twice
for rep in 1 2; do
for so in build_variants/*.so; do
  n=$(basename $so .so)
  IMPALA_HIP_LIB=$so timeout -k 10 120 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-host-staged --no-fp32-line > gpurun_out/vb_$n.json 2>/dev/null || { echo "variant $n: exit $?"; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/vb_$n.json').read().strip().splitlines()[-1]); print('$n', d['ms_per_step'], d['kernel_us'])"
done
done
