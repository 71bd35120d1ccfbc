#!/bin/bash
# quick fp32 check: launch-mode / parity tests of the step kernels, then the default bench line
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/quick32
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q -s --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_parity_full.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python bench.py --no-cpu-baseline --no-host-staged ${BENCH_ARGS:-} > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python - <<'PY'
import json
d = json.loads(open("gpurun_out/quick32/bench.json").read().strip().splitlines()[-1])
print(d["dtype"], d["value"], d["ms_per_step"], d["kernel_us"])
alt = d.get("bf16_mode") or d.get("fp32_parity_mode")
if alt: print(alt["dtype"], alt["value"], alt["ms_per_step"], alt["kernel_us"])
PY
