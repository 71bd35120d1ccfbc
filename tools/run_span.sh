#!/bin/bash
# stamp / span lines of each build_variants/*.so (bench run, last launch's lines)
for so in build_variants/*.so; do
  n=$(basename $so .so)
  IMPALA_HIP_LIB=$so timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-host-staged --no-fp32-line > gpurun_out/st_$n.log 2>&1 || echo "variant $n: exit $?"
  echo "== $n"; grep -E '^[A-Z0-9]+ ' gpurun_out/st_$n.log | tail -24
done
