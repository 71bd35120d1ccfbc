#!/bin/bash
# One rocprofv3 PMC pass (its own run, --kernel-trace only beside it) over the bench (fp32; BENCH_ARGS="--dtype bf16" for bf16):
# effective clock (GRBM_GUI_ACTIVE / 8 / duration), MFMA busy cycles, wave cycles, LDS bank
# conflicts per learner kernel.  tools/pmc_util.py summarises gpurun_out/<tag>/pmc.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r04pmc}
mkdir -p $O
timeout -s KILL 240 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-trace --output-format csv -d $O/pmc -o run -- python3 bench.py --steps 20 --warmup 20 --settle-ms 0 --no-cpu-baseline --no-host-staged --no-alt-line --no-dp-variants --no-learner-loop --no-actor-act ${BENCH_ARGS:-} > $O/bench.json 2> $O/pmc.err || { echo "pmc rc=$?"; tail -5 $O/pmc.err; exit 1; }
python3 tools/pmc_util.py $O/pmc | tee $O/pmc_util.txt
