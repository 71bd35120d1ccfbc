#!/bin/bash
# Round 5, call C: the copy-path priming in impala_stage_init (hs_calls.py, fresh processes,
# primed and IMPALA_STAGE_PRIME=0), then the driver's bench command twice with --settle-ms.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05c
mkdir -p $O
for i in 1 2; do
  timeout -k 10 200 python3 tools/hs_calls.py 5 20 > $O/hs_primed$i.txt 2>&1 || { echo "hs rc=$?"; tail $O/hs_primed$i.txt; exit 1; }
done
IMPALA_STAGE_PRIME=0 timeout -k 10 200 python3 tools/hs_calls.py 5 20 > $O/hs_noprime.txt 2>&1 || { echo "hs0 rc=$?"; exit 1; }
for i in 1 2; do
  timeout -k 10 240 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/b$i.json 2> $O/b$i.err || { echo "bench $i rc=$?"; tail -20 $O/b$i.err; exit 1; }
done
echo done
