#!/bin/bash
# Round 6 (gpurun_out/r06r/): the staging block's host allocation flags
# (IMPALA_STAGE_HOSTMEM=1: mapped + portable; 0: default) for the host-list loop, three
# processes each, interleaved.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06r
mkdir -p $O
fatal() { case $1 in 124|137|134|139) echo "fatal rc=$1 in $2"; exit 1;; esac; }
Q="--steps 20 --warmup 5 --no-alt-line --no-cpu-baseline"
for i in 1 2 3; do
for v in 0 1; do
  IMPALA_STAGE_HOSTMEM=$v timeout -k 10 300 python bench.py $Q > $O/hm$v$i.json 2> $O/hm$v$i.err; rc=$?; fatal $rc hm$v$i
  python3 -c "import json;d=json.load(open('$O/hm$v$i.json'));l=d['learner_loop']['host_list_replay'];print('hostmem $v run $i', 'hs', d['host_staged']['ms_per_step'], 'list', {k:(v['ms_per_step'],v['ms_per_step_median'],v['host_ms_per_iter_median']) for k,v in l.items()})"
done
done
