#!/bin/bash
# PPO and SAC bench lines (bf16 + fp32 PPO), gpurun_out/algos/
set -o pipefail
O=gpurun_out/algos
mkdir -p $O
timeout -k 10 200 python bench.py --algo ppo --no-host-staged > $O/ppo_bf16.json 2> $O/ppo_bf16.err || exit $?
timeout -k 10 200 python bench.py --algo ppo --dtype fp32 --no-cpu-baseline --no-host-staged > $O/ppo_fp32.json 2> $O/ppo_fp32.err || exit $?
timeout -k 10 200 python bench.py --algo sac --steps 200 --warmup 20 --cpu-seconds 12 > $O/sac_bf16.json 2> $O/sac_bf16.err || exit $?
for f in $O/*.json; do python -c "
import json,sys
d=json.loads(open('$f').read().strip().splitlines()[-1])
print('$f', d['value'], d['unit'], d['ms_per_step'], (d.get('cpu_baseline') or {}).get('value'), d.get('kernel_us'))
"; done
