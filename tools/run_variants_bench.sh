#!/bin/bash
# bench.py ms/step and per-kernel us of each build_variants/*.so, interleaved twice (same box)
for r in 1 2; do
  for so in build_variants/*.so; do
    n=$(basename $so .so)
    IMPALA_HIP_LIB=$so timeout -k 10 120 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-host-staged --no-fp32-line "$@" 2>/dev/null > gpurun_out/var_$n.json || { echo "$n failed"; continue; }
    python - "$n" <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/var_{sys.argv[1]}.json").read().strip().splitlines()[-1])
k = d["kernel_us"]
print(f"{sys.argv[1]:10s} {d['ms_per_step']:.4f} ms  " + " ".join(f"{a}={b}" for a, b in k.items()))
PY
  done
done
