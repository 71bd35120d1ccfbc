#!/bin/bash
# Round 5, call E: copy-path priming with all rounds in flight -- hs_calls.py in fresh
# processes, its HSA API trace (long hsa_amd_memory_async_copy_on_engine calls), the bench.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05e}
mkdir -p $O
for i in 1 2; do
  timeout -k 10 200 python3 tools/hs_calls.py 5 20 > $O/hs_primed$i.txt 2>&1 || { echo "hs rc=$?"; tail $O/hs_primed$i.txt; exit 1; }
done
timeout -k 10 240 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/b1.json 2> $O/b1.err || { echo "bench rc=$?"; tail -20 $O/b1.err; exit 1; }
cd /tmp
timeout -k 10 300 rocprofv3 --hip-runtime-trace --hsa-trace -d $GRAFT_REPO_ROOT/$O/api -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/hs_calls.py 5 20 > $GRAFT_REPO_ROOT/$O/hs_api.txt 2>&1 || { echo "trace rc=$?"; tail $GRAFT_REPO_ROOT/$O/hs_api.txt; exit 1; }
echo done
