#!/bin/bash
# Round 4: bench lines of the product library and every build_variants/*.so (A/B, stamps), then
# the parity files verbose, the whole -m gpu suite and smoke().  Stop at the first failure.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r04f}
mkdir -p $O
for so in build_variants/*.so; do
  n=$(basename $so .so)
  IMPALA_HIP_LIB=$PWD/$so timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-host-staged --no-alt-line > $O/vb_$n.json 2> $O/vb_$n.err || { echo "variant $n rc=$?"; tail -5 $O/vb_$n.err; exit 1; }
  grep -aE '^[A-Z0-9]+ ' $O/vb_$n.json | tail -2 || true
  python -c "import json; d=json.loads([l for l in open('$O/vb_$n.json') if l.startswith('{')][-1]); print('$n', d['ms_per_step'], d['kernel_us'])"
done
timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-host-staged --no-alt-line > $O/vb_product.json 2>/dev/null && python -c "import json; d=json.loads([l for l in open('$O/vb_product.json') if l.startswith('{')][-1]); print('product', d['ms_per_step'], d['kernel_us'])"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity_full.py tests/test_gpu_parity.py -v -s -m gpu --timeout 300 --timeout-method thread > $O/parity.log 2>&1 || { echo "parity rc=$?"; grep -E "FAIL|Error|assert" $O/parity.log | head -40; tail -5 $O/parity.log; exit 1; }
tail -1 $O/parity.log
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -30 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
