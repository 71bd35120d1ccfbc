#!/bin/bash
# Round 4: bench lines (200 steps, fp32 C2) of the product and every build_variants/*.so,
# product first and last (box drift); variants that print stamp lines show them.
set -o pipefail
shopt -s nullglob
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r04v}
mkdir -p $O
bl() {  # name, lib
  IMPALA_HIP_LIB=$2 timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-host-staged --no-alt-line --no-dp-variants > $O/vb_$1.json 2> $O/vb_$1.err || { echo "bench $1 rc=$?"; tail -5 $O/vb_$1.err; exit 1; }
  grep -aE '^[A-Z0-9]+ ' $O/vb_$1.json | tail -2 || true
  python -c "import json; d=json.loads([l for l in open('$O/vb_$1.json') if l.startswith('{')][-1]); print('$1', d['ms_per_step'], d['kernel_us'])"
}
bl product $PWD/impala_amd/libimpala_hip.so
for so in build_variants/*.so; do bl $(basename $so .so) $PWD/$so; done
bl product2 $PWD/impala_amd/libimpala_hip.so
