#!/bin/bash
# Round 6 (gpurun_out/$TAG/): the A/B library's launch merges against the default launches on
# the final tree, both dtypes (bench.py headline in that dtype, 100 steps): the slab reduction
# + clip + Adam in one launch (IMPALA_FUSED_UPDATE=1) and early reduction of the final slabs
# inside the conv weight-gradient launch (IMPALA_EARLY_RED=1).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06fu}
mkdir -p $O
export IMPALA_HIP_LIB=$PWD/impala_amd/libimpala_hip_ab.so
ARGS="--steps 100 --warmup 20 --no-cpu-baseline --no-host-staged --no-learner-loop --no-alt-line"
for dt in fp32 bf16; do
for v in default FUSED_UPDATE EARLY_RED default; do
  if [ $v = default ]; then E=""; else E="IMPALA_$v=1"; fi
  env $E timeout -k 10 300 python bench.py --dtype $dt $ARGS > $O/b_${dt}_$v.json 2> $O/b_${dt}_$v.err || { echo "rc=$? at $dt $v"; tail -5 $O/b_${dt}_$v.err; exit 1; }
  python3 - $O/b_${dt}_$v.json "$dt $v" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print(sys.argv[2], d["ms_per_step"], d["ms_per_step_median"], {k: round(v, 2) for k, v in d.get("kernel_us", {}).items()})
PY
done
done
