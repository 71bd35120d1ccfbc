#!/bin/bash
# Round 6 (gpurun_out/r06n/): the host-list loop with the staging threads pinned to the learner
# thread's NUMA node (default) or not (IMPALA_STAGE_PIN=0), three processes each, interleaved.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06n
mkdir -p $O
fatal() { case $1 in 124|137|134|139) echo "fatal rc=$1 in $2"; exit 1;; esac; }
Q="--steps 20 --warmup 5 --no-alt-line --no-cpu-baseline"
python3 -c "import os; print('cpus', len(os.sched_getaffinity(0)), 'nodes', sorted(os.listdir('/sys/devices/system/node')))"
for i in 1 2 3; do
for v in pin:1 nopin:0; do
  name=${v%%:*}; p=${v#*:}
  IMPALA_STAGE_PIN=$p timeout -k 10 300 python bench.py $Q > $O/${name}$i.json 2> $O/${name}$i.err; rc=$?; fatal $rc $name$i
  python3 -c "import json;d=json.load(open('$O/${name}$i.json'));l=d['learner_loop']['host_list_replay'];print('$name$i', 'hs', d['host_staged']['ms_per_step'], 'list', {k:(v['ms_per_step'],v['ms_per_step_median']) for k,v in l.items()})"
done
done
