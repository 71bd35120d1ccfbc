#!/bin/bash
# A/B of the product library against build_variants/$1.so (and optional more variants):
# bench.py --steps 100 interleaved twice, per-kernel us.  usage: tools/r05_ab.sh <tag> old [more...]
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/$1; shift
mkdir -p $O
for r in 1 2; do
  for n in product "$@"; do
    if [ $n = product ]; then unset IMPALA_HIP_LIB; else export IMPALA_HIP_LIB=build_variants/$n.so; fi
    timeout -k 10 120 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-host-staged --no-alt-line $BENCH_ARGS > $O/$n.$r.json 2> $O/$n.$r.err || { echo "$n failed"; tail -5 $O/$n.$r.err; exit 1; }
    python -c "
import json,sys; d=json.loads(open('$O/$n.$r.json').read().strip().splitlines()[-1]); k=d['kernel_us']
print('$n', d['ms_per_step'], d['ms_per_step_median'], ' '.join(f'{a}={b}' for a,b in k.items()))"
  done
done
