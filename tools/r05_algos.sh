#!/bin/bash
# PPO and SAC bench lines (BASELINE configs 4 and 5) on this tree, both dtypes, 100 steps.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r05alg}
mkdir -p $O
for a in ppo sac; do
  for dt in bf16 fp32; do
    timeout -k 10 300 python bench.py --algo $a --dtype $dt --steps 100 --warmup 10 --no-cpu-baseline --no-host-staged --no-alt-line > $O/$a.$dt.json 2> $O/$a.$dt.err || { echo "$a $dt failed"; tail -5 $O/$a.$dt.err; exit 1; }
    python -c "
import json; d=json.loads(open('$O/$a.$dt.json').read().strip().splitlines()[-1])
print('$a $dt', d['value'], d['unit'], d['ms_per_step'], d.get('ms_per_step_median'))"
  done
done
