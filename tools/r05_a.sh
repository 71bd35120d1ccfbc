#!/bin/bash
# Round 5, call A: the driver's bench command (--steps 20 --warmup 5) three times in fresh
# processes with per-step event times, then once under a kernel + memory-copy trace.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05a
mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 240 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/b$i.json 2> $O/b$i.err || { echo "bench $i rc=$?"; tail -20 $O/b$i.err; exit 1; }
  echo "bench $i done"
done
timeout -k 10 240 python3 bench.py --gpus 1 --steps 100 --warmup 10 --no-cpu-baseline > $O/b100.json 2> $O/b100.err || { echo "bench100 rc=$?"; tail -20 $O/b100.err; exit 1; }
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $GRAFT_REPO_ROOT/$O/trace -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $GRAFT_REPO_ROOT/$O/btrace.json 2> $GRAFT_REPO_ROOT/$O/btrace.err || { echo "trace rc=$?"; tail -20 $GRAFT_REPO_ROOT/$O/btrace.err; exit 1; }
echo done
