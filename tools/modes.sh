#!/bin/bash
# launch modes of the IMPALA step: default, hipGraph replay, side stream for the wgrad branches
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/modes
mkdir -p $O
timeout -k 10 200 python bench.py --steps 200 --no-cpu-baseline --no-host-staged > $O/default.json 2> $O/default.err || exit $?
IMPALA_GRAPH=1 timeout -k 10 200 python bench.py --steps 200 --no-cpu-baseline --no-host-staged > $O/graph.json 2> $O/graph.err || exit $?
IMPALA_SIDE_STREAM=1 timeout -k 10 200 python bench.py --steps 200 --no-cpu-baseline --no-host-staged > $O/side.json 2> $O/side.err || exit $?
IMPALA_GRAPH=1 IMPALA_SIDE_STREAM=1 timeout -k 10 200 python bench.py --steps 200 --no-cpu-baseline --no-host-staged > $O/graph_side.json 2> $O/graph_side.err || exit $?
