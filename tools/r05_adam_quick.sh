#!/bin/bash
# Bitwise A/B of the product against build_variants/$BASE.so, then bench A/B fp32 + bf16.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r05aq}
mkdir -p $O
IMPALA_HIP_LIB=build_variants/$BASE.so timeout -k 10 120 python tools/bitwise_ab.py save $O/pre.npz > $O/bw.txt 2>&1 || { echo "save pre rc=$?"; tail $O/bw.txt; exit 1; }
timeout -k 10 120 python tools/bitwise_ab.py save $O/new.npz >> $O/bw.txt 2>&1 || { echo "save new rc=$?"; tail $O/bw.txt; exit 1; }
python tools/bitwise_ab.py cmp $O/pre.npz $O/new.npz | tee -a $O/bw.txt || exit 1
rm -f $O/pre.npz $O/new.npz
bash tools/r05_ab.sh ${1:-r05aq}/ab $BASE || exit 1
BENCH_ARGS="--dtype bf16" bash tools/r05_ab.sh ${1:-r05aq}/abb $BASE || exit 1
