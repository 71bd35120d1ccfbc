#!/bin/bash
# The FC-row Adam (adam_kernel re-emits the FC weight's kernel-layout rows through LDS):
# bitwise A/B against the previous build (build_variants/${BASE:-pre_adam}.so), the -m gpu suite, and
# bench A/B fp32 + bf16.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r05adam}
mkdir -p $O
IMPALA_HIP_LIB=build_variants/${BASE:-pre_adam}.so timeout -k 10 120 python tools/bitwise_ab.py save $O/pre.npz > $O/bw.txt 2>&1 || { echo "save pre rc=$?"; tail $O/bw.txt; exit 1; }
timeout -k 10 120 python tools/bitwise_ab.py save $O/new.npz >> $O/bw.txt 2>&1 || { echo "save new rc=$?"; tail $O/bw.txt; exit 1; }
python tools/bitwise_ab.py cmp $O/pre.npz $O/new.npz | tee -a $O/bw.txt || exit 1
rm -f $O/pre.npz $O/new.npz
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash tools/r05_ab.sh ${1:-r05adam}/ab ${BASE:-pre_adam} || exit 1
BENCH_ARGS="--dtype bf16" bash tools/r05_ab.sh ${1:-r05adam}/abb ${BASE:-pre_adam} || exit 1
