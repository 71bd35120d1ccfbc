#!/bin/bash
# bench.py ms/step of each build_variants/*.so, interleaved twice (same box, same clocks)
for r in 1 2; do
  for so in build_variants/*.so; do
    n=$(basename $so .so)
    IMPALA_HIP_LIB=$so timeout -k 10 120 python bench.py --steps 300 --warmup 20 --no-cpu-baseline --roofline-kernel adam 2>/dev/null | python -c "import json,sys; print('$n', json.loads(sys.stdin.read())['ms_per_step'])" || echo "$n failed"
  done
done
