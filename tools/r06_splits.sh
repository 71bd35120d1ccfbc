#!/bin/bash
# Round 6 (gpurun_out/$TAG/): the conv weight gradients' split counts (IMPALA_WG3_TARGET /
# IMPALA_WG2_TARGET, default 256 / 256) against the step, both dtypes: bench.py headline + bf16
# line only (no loop, host staging, CPU baseline).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06sp}
mkdir -p $O
ARGS="--steps 100 --warmup 20 --no-cpu-baseline --no-host-staged --no-learner-loop"
for cfg in 256:256 128:128 256:128 128:256 512:512 256:256; do
  w3=${cfg%%:*}; w2=${cfg##*:}
  IMPALA_WG3_TARGET=$w3 IMPALA_WG2_TARGET=$w2 timeout -k 10 300 python bench.py $ARGS > $O/b_${w3}_${w2}.json 2> $O/b_${w3}_${w2}.err || { echo "rc=$? at $cfg"; tail -5 $O/b_${w3}_${w2}.err; exit 1; }
  python3 - $O/b_${w3}_${w2}.json $cfg <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print(sys.argv[2], "fp32", d["ms_per_step"], d["ms_per_step_median"], "bf16", d["bf16_mode"]["ms_per_step"], d["bf16_mode"].get("ms_per_step_median"))
PY
done
