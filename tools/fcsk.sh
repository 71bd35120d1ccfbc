#!/bin/bash
# fp32 FC forward variants (IMPALA_FC_SPLITK: 0 = 32x32 tiles, 1 = split-K over workgroups with
# an in-launch combine, 2 = K split over the waves of a workgroup): the -m gpu suite under the
# variant in $V, then the bench for each variant
set -o pipefail
export TMPDIR=/tmp
# the variants live in the A/B build only (python -m impala_amd.build --ab)
export IMPALA_HIP_LIB=impala_amd/libimpala_hip_ab.so
O=gpurun_out/fcsk
V=${V:-2}
mkdir -p $O
IMPALA_FC_SPLITK=$V timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for f in 2 0 2 0; do
  IMPALA_FC_SPLITK=$f timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_$f.json 2> $O/bench_$f.err || exit $?
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], d.get('kernel_us'))" $O/bench_$f.json $f
done
