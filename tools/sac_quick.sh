set -o pipefail
export TMPDIR=/tmp
timeout -k 10 120 python -u -m pytest tests/test_gpu_sac.py -x -q --timeout 120 --timeout-method thread > gpurun_out/sac_t.log 2>&1 || exit $?
IMPALA_HIP_LIB=build_variants/sacstamps.so timeout -k 10 120 python bench.py --algo sac --steps 20 --warmup 5 --no-cpu-baseline --roofline-kernel critic_fwd_chain > gpurun_out/stamps.log 2>&1
timeout -k 10 120 python bench.py --algo sac --steps 300 --warmup 20 --no-cpu-baseline > gpurun_out/sac_b.json 2>gpurun_out/sac_b.err || exit $?
