#!/bin/bash
# H2D copy-stream count for the host-staged pass (1 vs 4 vs 8), then the SAC PMC traffic passes.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/stage
mkdir -p $O
for n in 1 4 8; do
  IMPALA_H2D_STREAMS=$n timeout -k 10 200 python bench.py --steps 50 --warmup 5 --no-cpu-baseline > $O/staged$n.json 2> $O/staged$n.err || exit $?
done
bash tools/profile.sh r01k_sac --algo sac --roofline-kernel actor_chain
