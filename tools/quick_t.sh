#!/bin/bash
# selected GPU tests (args = pytest -k expression), then the quick bench line
set -o pipefail
O=gpurun_out/quick
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$1" > $O/tests_k.log 2>&1 || { tail -30 $O/tests_k.log; exit 1; }
tail -2 $O/tests_k.log
shift
timeout -k 10 300 python bench.py --no-cpu-baseline --no-host-staged --no-fp32-line "$@" > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python - <<'PY'
import json
d = json.loads(open("gpurun_out/quick/bench.json").read().strip().splitlines()[-1])
print("ms/step", d["ms_per_step"], "value", d["value"])
print("kernel_us", d["kernel_us"])
PY
