#!/bin/bash
# printf stamp lines of one build_variants/<name>.so: all of them (grouped by prefix)
so=build_variants/$1.so
IMPALA_HIP_LIB=$so timeout -k 10 120 python bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-host-staged --no-fp32-line > gpurun_out/st_$1.log 2>&1 || echo "variant $1: exit $?"
grep -E '^[A-Z0-9]+ ' gpurun_out/st_$1.log | sort | uniq | head -80
