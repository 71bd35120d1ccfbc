#!/bin/bash
# quick GPU check after a kernel change: the -m gpu suite, then the bench line without the CPU
# and host-staged legs (gpurun_out/quick/)
set -o pipefail
O=gpurun_out/quick
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python bench.py --no-cpu-baseline --no-host-staged "$@" > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python - <<'PY'
import json
d = json.loads(open("gpurun_out/quick/bench.json").read().strip().splitlines()[-1])
print("ms/step", d["ms_per_step"], "value", d["value"])
print("kernel_us", d["kernel_us"])
f = d.get("fp32_parity_mode")
if f: print("fp32 ms/step", f["ms_per_step"], f["kernel_us"])
PY
