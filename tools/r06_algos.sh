#!/bin/bash
# Round 6 (gpurun_out/$TAG/): bench.py's other lines on the current tree -- the data-parallel
# path at world size 1 over RCCL (IMPALA_BENCH_DIST=1: barriers, max over ranks, dp_variants),
# then the PPO and SAC learners.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06v2}
mkdir -p $O
RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29571 IMPALA_BENCH_DIST=1 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_dist1.json 2> $O/bench_dist1.err || exit $?
timeout -k 10 300 python bench.py --algo ppo --steps 50 --warmup 10 --no-cpu-baseline > $O/bench_ppo.json 2> $O/bench_ppo.err || exit $?
timeout -k 10 300 python bench.py --algo sac --steps 50 --warmup 10 --no-cpu-baseline > $O/bench_sac.json 2> $O/bench_sac.err || exit $?
for f in dist1 ppo sac; do
python3 - $O/bench_$f.json $f <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
dv = {k: (v.get("ms_per_step"), v.get("replicas_bitwise_equal"), v.get("bitwise_equal_to_c10d_1bucket"))
      for k, v in d.get("dp_variants", {}).items() if isinstance(v, dict)}
print(sys.argv[2], d["value"], d["ms_per_step"], d["dtype"], d["config"].get("allreduce"), dv)
PY
done
