#!/bin/bash
# Round 5, call H: weight-gradient operand-traffic knock-outs (tools/var_specs/wgl2.py)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05h
mkdir -p $O
for r in 1 2; do
  for n in wl_base wl_x wl_y wl_xy; do
    IMPALA_HIP_LIB=build_variants/$n.so timeout -k 10 120 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-host-staged --no-alt-line > $O/$n.$r.json 2> $O/$n.$r.err || { echo "$n failed"; tail -5 $O/$n.$r.err; exit 1; }
    python -c "
import json,sys; d=json.loads(open('$O/$n.$r.json').read().strip().splitlines()[-1]); k=d['kernel_us']
print('$n', d['ms_per_step'], ' '.join(f'{a}={b}' for a,b in k.items()))"
  done
done
