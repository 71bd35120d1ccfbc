#!/bin/bash
# Round 4: the fp32 step with the FC weight gradient written straight into the gradient
# (IMPALA_FC_DIRECT=1: no FC slab in fc_bwd or reduce_grads) against the split-slab default.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r04fcd}
mkdir -p $O
for v in 0 1 0 1; do
  IMPALA_FC_DIRECT=$v timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-host-staged --no-alt-line --no-dp-variants > $O/fcd$v.json 2> $O/fcd$v.err || { echo "bench rc=$?"; tail -5 $O/fcd$v.err; exit 1; }
  python -c "import json; d=json.loads([l for l in open('$O/fcd$v.json') if l.startswith('{')][-1]); print('fc_direct=$v', d['ms_per_step'], d['kernel_us'])"
done
