#!/bin/bash
# Round 4: host-staged copy paths, second pass -- hipMemcpyAsync (SDMA) on 1 / 2 / 4 copy
# streams and the pull kernel at 64 / 128 threads per workgroup, each alone and beside the fp32
# step (tools/h2d_bw.py), then bench.py's host_staged record for the default path.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r04hs2}
mkdir -p $O
run() {
  env "$@" timeout -k 10 120 python tools/h2d_bw.py 40 >> $O/h2d_bw.txt 2>&1 || { echo "h2d_bw $* rc=$?"; tail -5 $O/h2d_bw.txt; exit 1; }
  echo "  ^ $*" >> $O/h2d_bw.txt
}
run IMPALA_H2D_KERNEL=0 IMPALA_H2D_STREAMS=1
run IMPALA_H2D_KERNEL=0 IMPALA_H2D_STREAMS=2
run IMPALA_H2D_KERNEL=0 IMPALA_H2D_STREAMS=4
run IMPALA_H2D_KERNEL=8 IMPALA_H2D_THREADS=64
run IMPALA_H2D_KERNEL=16 IMPALA_H2D_THREADS=128
run IMPALA_H2D_KERNEL=8
grep -A1 "H2D path" $O/h2d_bw.txt
timeout -k 10 300 python bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-alt-line --no-dp-variants > $O/bench.json 2> $O/bench.err || { echo "bench rc=$?"; tail -5 $O/bench.err; exit 1; }
python -c "import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print(d['value'], d.get('host_staged'))"
