#!/bin/bash
# Round 6 (gpurun_out/r06p/): the host-list loop with 8 / 16 staging pool threads
# (IMPALA_STAGE_THREADS), three processes each, interleaved (prefetch 2).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06p
mkdir -p $O
fatal() { case $1 in 124|137|134|139) echo "fatal rc=$1 in $2"; exit 1;; esac; }
Q="--steps 20 --warmup 5 --no-alt-line --no-cpu-baseline"
for i in 1 2 3; do
for t in 8 16 24; do
  IMPALA_STAGE_THREADS=$t timeout -k 10 300 python bench.py $Q > $O/t${t}_$i.json 2> $O/t${t}_$i.err; rc=$?; fatal $rc t$t
  python3 -c "import json;d=json.load(open('$O/t${t}_$i.json'));l=d['learner_loop']['host_list_replay'];print('t$t run $i', 'hs', d['host_staged']['ms_per_step'], 'list', {k:(v['ms_per_step'],v['ms_per_step_median'],v['host_ms_per_iter_median']) for k,v in l.items()})"
done
done
