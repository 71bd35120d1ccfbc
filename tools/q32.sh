#!/bin/bash
# quick fp32 check after a kernel change (gpurun_out/q32/): the -m gpu suite, then the bench line
# without the CPU / host-staged legs (fp32 headline + bf16 sub-record)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/q32
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread ${TESTS:-} > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python bench.py --no-cpu-baseline --no-host-staged "$@" > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python - <<'PY'
import json
d = json.loads(open("gpurun_out/q32/bench.json").read().strip().splitlines()[-1])
print(d["dtype"], "ms/step", d["ms_per_step"], "value", d["value"], "frac", d["roofline"]["frac"])
print("kernel_us", d["kernel_us"])
b = d.get("bf16_mode") or d.get("fp32_parity_mode")
if b: print(b["dtype"], "ms/step", b["ms_per_step"], b["kernel_us"])
PY
