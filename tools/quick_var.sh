set -o pipefail
mkdir -p gpurun_out/quick
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/quick/tests.log 2>&1 || { tail -30 gpurun_out/quick/tests.log; exit 1; }
tail -2 gpurun_out/quick/tests.log
bash tools/run_variants_bench.sh
