#!/bin/bash
# fp32 bf16 FC backward at two workgroups per CU: bitwise against
# build_variants/pre_fcbb.so, the parity files, bench A/B.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r05fcbb2}
mkdir -p $O
IMPALA_HIP_LIB=build_variants/pre_fcbb.so timeout -k 10 120 python tools/bitwise_ab.py save $O/pre.npz > $O/bw.txt 2>&1 || { echo "save pre rc=$?"; tail $O/bw.txt; exit 1; }
timeout -k 10 120 python tools/bitwise_ab.py save $O/new.npz >> $O/bw.txt 2>&1 || { echo "save new rc=$?"; tail $O/bw.txt; exit 1; }
python tools/bitwise_ab.py cmp $O/pre.npz $O/new.npz | tee -a $O/bw.txt
rm -f $O/pre.npz $O/new.npz
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_parity_full.py -x -q -m gpu --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
BENCH_ARGS="--dtype bf16" bash tools/r05_ab.sh ${1:-r05fcbb2}/ab pre_fcbb || exit 1
