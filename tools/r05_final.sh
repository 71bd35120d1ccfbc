#!/bin/bash
# Round 5 rehearsal of the driver's round-end commands on this tree (gpurun_out/r05final/):
# pytest -m gpu, smoke(), the driver's bench command twice, then rocprofv3 stats + HBM counters
# of the fp32 and bf16 steps (tools/profile.sh).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${OTAG:-r05final}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for i in 1 2; do
  timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench$i.json 2> $O/bench$i.err || { echo "bench rc=$?"; tail -20 $O/bench$i.err; exit 1; }
done
bash tools/profile.sh ${PTAG:-r05f32} || { echo "profile fp32 rc=$?"; exit 1; }
bash tools/profile.sh ${PTAG:-r05f32}b --dtype bf16 || { echo "profile bf16 rc=$?"; exit 1; }
echo done
