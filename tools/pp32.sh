#!/bin/bash
# fp32 conv12 backward A/B: parity tests, then the bench line with the fused / split launch
set -o pipefail
export TMPDIR=/tmp
bash tools/quick32.sh || exit 1
for lc in 0 1; do
  IMPALA_LC12=$lc timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-host-staged --no-fp32-line > gpurun_out/lc$lc.json 2>/dev/null || exit $?
  python -c "import json; d=json.loads(open('gpurun_out/lc$lc.json').read().strip().splitlines()[-1]); print('lc12=$lc', d['ms_per_step'], d['kernel_us'])"
done
