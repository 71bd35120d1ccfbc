#!/bin/bash
# PPO / SAC bench lines, both dtypes, on the current tree -> gpurun_out/r04alg/
set -o pipefail
mkdir -p gpurun_out/r04alg
for a in ppo sac; do
  for d in fp32 bf16; do
    timeout -k 10 300 python bench.py --algo $a --dtype $d --steps 300 --warmup 30 --no-cpu-baseline \
      > gpurun_out/r04alg/${a}_${d}.json 2> gpurun_out/r04alg/${a}_${d}.err || exit $?
  done
done
python - <<'PY'
import json
for a in ("ppo", "sac"):
    for d in ("fp32", "bf16"):
        x = json.loads(open(f"gpurun_out/r04alg/{a}_{d}.json").read().strip().splitlines()[-1])
        print(a, d, x["value"], x["ms_per_step"], x["dtype"])
PY
