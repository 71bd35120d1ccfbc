#!/bin/bash
# Direct launches against hipGraph replay of whole steps (IMPALA_GRAPH=1), fp32 and bf16:
# bench.py --steps 100 interleaved twice.  Then the launch-boundary probe (tools/probe/launch_floor).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r05gr}
mkdir -p $O
timeout -k 10 120 ./tools/probe/launch_floor > $O/launch_floor.txt 2>&1 || { echo "probe rc=$?"; exit 1; }
cat $O/launch_floor.txt
for r in 1 2; do
  for dt in fp32 bf16; do
    for g in 0 1; do
      n=$dt.g$g.$r
      IMPALA_GRAPH=$g timeout -k 10 120 python bench.py --steps 100 --warmup 10 --dtype $dt --no-cpu-baseline --no-host-staged --no-alt-line > $O/$n.json 2> $O/$n.err || { echo "$n failed"; tail -5 $O/$n.err; exit 1; }
      python -c "
import json; d=json.loads(open('$O/$n.json').read().strip().splitlines()[-1])
print('$n', d['ms_per_step'], d['ms_per_step_median'], d['ms_per_step_max'])"
    done
  done
done
