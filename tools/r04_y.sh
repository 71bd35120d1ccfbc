#!/bin/bash
# Round 4: row-stride probe, then bench lines (200 steps) of the product and every
# build_variants/*.so, product first and last (box drift).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r04y}
mkdir -p $O
timeout -k 10 120 tools/probe/rowstride > $O/rowstride.txt 2>&1 || { echo "probe rc=$?"; tail -5 $O/rowstride.txt; exit 1; }
cat $O/rowstride.txt
bl() {  # name, lib
  IMPALA_HIP_LIB=$2 timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-host-staged --no-alt-line --no-dp-variants > $O/vb_$1.json 2> $O/vb_$1.err || { echo "bench $1 rc=$?"; tail -5 $O/vb_$1.err; exit 1; }
  python -c "import json; d=json.loads([l for l in open('$O/vb_$1.json') if l.startswith('{')][-1]); print('$1', d['ms_per_step'], d['kernel_us'])"
}
bl product $PWD/impala_amd/libimpala_hip.so
for so in build_variants/*.so; do bl $(basename $so .so) $PWD/$so; done
bl product2 $PWD/impala_amd/libimpala_hip.so
