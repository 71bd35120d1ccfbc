#!/bin/bash
# bench.py ms/step and per-kernel us under a few runtime environment settings, interleaved twice
set -o pipefail
run() {
  env "$@" timeout -k 10 120 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-host-staged --no-fp32-line 2>/dev/null > gpurun_out/envab.json || { echo "$* failed"; return; }
  python - "$*" <<'PY'
import json, sys
d = json.loads(open("gpurun_out/envab.json").read().strip().splitlines()[-1])
print(f"{sys.argv[1]:40s} {d['ms_per_step']:.4f} ms  " + " ".join(f"{a}={b}" for a, b in d["kernel_us"].items()))
PY
}
SETS=${ENV_SETS:-"X=base HIP_FORCE_DEV_KERNARG=0 IMPALA_GRAPH=1"}
for r in 1 2; do
  for e in $SETS; do run $e; done
done
