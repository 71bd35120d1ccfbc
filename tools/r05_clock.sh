#!/bin/bash
# The device step clock: its GPU tests, the instrumentation A/B (tools/region_order.py: event
# per step / device clock / unmarked), the driver's bench command twice, and the data-parallel
# bench path at world size 1 under torch.distributed.run (IMPALA_BENCH_DIST=1).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r05clk}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v -m gpu -k "step_clock or deterministic or launch_modes" --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 120 python tools/region_order.py fp32 > $O/region_order_fp32.txt 2>&1 || { echo "ro rc=$?"; tail $O/region_order_fp32.txt; exit 1; }
timeout -k 10 120 python tools/region_order.py bf16 > $O/region_order_bf16.txt 2>&1 || { echo "ro rc=$?"; tail $O/region_order_bf16.txt; exit 1; }
cat $O/region_order_fp32.txt $O/region_order_bf16.txt
for i in 1 2; do
  timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench$i.json 2> $O/bench$i.err || { echo "bench rc=$?"; tail -20 $O/bench$i.err; exit 1; }
  python -c "
import json; d=json.loads(open('$O/bench$i.json').read().strip().splitlines()[-1])
hs=d['host_staged']; b=d['bf16_mode']
print('fp32', d['value'], d['ms_per_step'], d['ms_per_step_median'], d['ms_per_step_max'], d['steps_sum_ms'])
print('bf16', b['value'], b['ms_per_step'], b['ms_per_step_median'], b['ms_per_step_max'])
print('hs', hs['value'], hs['ms_per_step'], hs['ms_per_step_median'], hs['ms_per_step_max'])"
done
IMPALA_BENCH_DIST=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_dist.json 2> $O/bench_dist.err || { echo "dist rc=$?"; tail -20 $O/bench_dist.err; exit 1; }
python -c "
import json; d=json.loads(open('$O/bench_dist.json').read().strip().splitlines()[-1])
print('dist', d['value'], d['ms_per_step'], d['ms_per_step_median'], d['config'].get('allreduce'), str(d.get('dp_variants'))[:400])"
