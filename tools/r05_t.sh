#!/bin/bash
# Round 5, call T: the driver's bench command on the final bench.py, plus the PPO and SAC lines.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05t
mkdir -p $O
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { echo "bench rc=$?"; tail -20 $O/bench.err; exit 1; }
timeout -k 10 300 python3 bench.py --algo ppo --steps 100 --warmup 10 --no-cpu-baseline > $O/ppo_fp32.json 2> $O/ppo.err || { echo "ppo rc=$?"; tail -20 $O/ppo.err; exit 1; }
timeout -k 10 300 python3 bench.py --algo ppo --dtype bf16 --steps 100 --warmup 10 --no-cpu-baseline --no-alt-line > $O/ppo_bf16.json 2>> $O/ppo.err || { echo "ppo bf16 rc=$?"; exit 1; }
timeout -k 10 300 python3 bench.py --algo sac --dtype bf16 --steps 100 --warmup 10 --no-cpu-baseline > $O/sac_bf16.json 2> $O/sac.err || { echo "sac rc=$?"; tail -20 $O/sac.err; exit 1; }
timeout -k 10 300 python3 bench.py --algo sac --dtype fp32 --steps 100 --warmup 10 --no-cpu-baseline > $O/sac_fp32.json 2>> $O/sac.err || { echo "sac fp32 rc=$?"; exit 1; }
echo done
