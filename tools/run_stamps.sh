#!/bin/bash
# printf stamp lines of each build_variants/*.so (tools/var_specs/*stamps*.py): last 10 per variant
for so in build_variants/*.so; do
  n=$(basename $so .so)
  echo "== $n"
  IMPALA_HIP_LIB=$so timeout -k 10 120 python bench.py --steps 30 --warmup 3 --no-cpu-baseline > gpurun_out/st_$n.log 2>&1 || echo "variant $n: exit $?"
  grep -v '^{' gpurun_out/st_$n.log | grep -E '^[A-Z0-9]+ ' | tail -10
done
