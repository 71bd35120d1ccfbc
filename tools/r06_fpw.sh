#!/bin/bash
# Round 6 (gpurun_out/$TAG/): frames per workgroup of the fused forward (IMPALA_C12F_FPW) and
# of the per-frame backward (IMPALA_C1_FPW), default cdiv(N, CUs) = 5 at N = 1280, against the
# bf16 and fp32 steps (bench.py headline in that dtype only).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06fpw}
mkdir -p $O
ARGS="--steps 100 --warmup 20 --no-cpu-baseline --no-host-staged --no-learner-loop --no-alt-line"
for dt in bf16 fp32; do
for cfg in 5:5 3:5 4:5 6:5 5:3 5:4 5:6 5:5; do
  f=${cfg%%:*}; c=${cfg##*:}
  IMPALA_C12F_FPW=$f IMPALA_C1_FPW=$c timeout -k 10 300 python bench.py --dtype $dt $ARGS > $O/b_${dt}_${f}_${c}.json 2> $O/b_${dt}_${f}_${c}.err || { echo "rc=$? at $dt $cfg"; tail -5 $O/b_${dt}_${f}_${c}.err; exit 1; }
  python3 - $O/b_${dt}_${f}_${c}.json "$dt $cfg" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print(sys.argv[2], d["ms_per_step"], d["ms_per_step_median"])
PY
done
done
