#!/bin/bash
# The tail kernels' floor: rocprofv3 durations of the launch probe's trivial kernels
# (tools/probe/launch_floor.hip), then the adam knock-outs (tools/var_specs/adamko.py) A/B.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r05tail}
mkdir -p $O
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/lf -o run --output-format csv -- ./tools/probe/launch_floor > $O/launch_floor.txt 2> $O/lf.err || { echo "probe rc=$?"; tail $O/lf.err; exit 1; }
cat $O/lf/run_kernel_stats.csv
bash tools/r05_ab.sh ${1:-r05tail}/ab adam_nosh adam_nonorm adam_both || exit 1
BENCH_ARGS="--dtype bf16" bash tools/r05_ab.sh ${1:-r05tail}/abb adam_nosh adam_both || exit 1
