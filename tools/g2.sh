set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/g2; mkdir -p $O
cat /proc/self/cgroup > $O/cgroup.txt; cat /sys/fs/cgroup/cpu.max >> $O/cgroup.txt 2>&1; nproc >> $O/cgroup.txt; lscpu >> $O/cgroup.txt 2>&1
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_learner.py tests/test_gpu_dp_c3.py tests/test_gpu_dp.py > $O/tests.log 2>&1 || { echo tests failed; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { echo bench failed; tail -20 $O/bench.err; exit 1; }
bash tools/profile.sh r03b > $O/prof.log 2>&1 || { echo prof failed; tail -20 $O/prof.log; exit 1; }
echo all ok
