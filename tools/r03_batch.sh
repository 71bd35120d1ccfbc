#!/bin/bash
set -o pipefail
bash tools/run_variants_bench.sh
for fu in 0 1; do
  IMPALA_FUSED_UPDATE=$fu timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-host-staged --no-fp32-line > gpurun_out/fu$fu.json 2>/dev/null || exit $?
  python -c "import json; d=json.loads(open('gpurun_out/fu$fu.json').read().strip().splitlines()[-1]); print('fused_update=$fu', d['ms_per_step'], d['kernel_us'])"
done
