#!/bin/bash
# Slab-reduction split loads per thread (impala.hip IMPALA_RED_LPT, default 16): bench A/B.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r05lpt}
mkdir -p $O
for r in 1 2; do
  for dt in fp32 bf16; do
    for l in 16 8 4; do
      n=$dt.l$l.$r
      IMPALA_RED_LPT=$l timeout -k 10 120 python bench.py --steps 100 --warmup 10 --dtype $dt --no-cpu-baseline --no-host-staged --no-alt-line > $O/$n.json 2> $O/$n.err || { echo "$n failed"; tail -3 $O/$n.err; exit 1; }
      python -c "
import json; d=json.loads(open('$O/$n.json').read().strip().splitlines()[-1]); k=d['kernel_us']
print('$n', d['ms_per_step'], d['ms_per_step_median'], 'reduce_grads', k['reduce_grads'], 'adam', k['adam'])"
    done
  done
done
