#!/bin/bash
# Round 5, call G: the -m gpu suite + smoke on this tree, then the bf16 step's rocprofv3 stats
# and HBM counters (tools/profile.sh r05bf --dtype bf16), and PMC utilisation passes (MFMA busy,
# effective clock, LDS conflicts) for bf16 and fp32.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05g
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 $O/smoke.log; exit 1; }
bash tools/profile.sh r05bf --dtype bf16 || { echo "profile rc=$?"; exit 1; }
TAG=r05g/pmc_bf16 BENCH_ARGS="--dtype bf16" bash tools/pmc_util.sh > /dev/null || { echo "pmc bf16 failed"; exit 1; }
TAG=r05g/pmc_fp32 bash tools/pmc_util.sh > /dev/null || { echo "pmc fp32 failed"; exit 1; }
echo done
