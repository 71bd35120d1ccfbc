set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/sac
timeout -k 10 200 python bench.py --algo sac --steps 200 --warmup 20 --cpu-seconds 12 > gpurun_out/sac/bench_bf16.json 2> gpurun_out/sac/bench_bf16.err || exit $?
timeout -k 10 200 python bench.py --algo sac --dtype fp32 --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/sac/bench_fp32.json 2> gpurun_out/sac/bench_fp32.err || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/sac/stats -o run --output-format csv -- python3 bench.py --algo sac --steps 50 --warmup 5 --no-cpu-baseline --roofline-kernel fwd_l2 > gpurun_out/sac/bench_stats.json 2> gpurun_out/sac/stats.err || exit $?
echo done
