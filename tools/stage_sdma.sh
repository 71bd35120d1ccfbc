#!/bin/bash
# host-staged pass: SDMA copies (default) vs blit-kernel copies (HSA_ENABLE_SDMA=0)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/stage
mkdir -p $O
timeout -k 10 200 python bench.py --steps 50 --warmup 5 --no-cpu-baseline > $O/staged_sdma.json 2> $O/staged_sdma.err || exit $?
HSA_ENABLE_SDMA=0 timeout -k 10 200 python bench.py --steps 50 --warmup 5 --no-cpu-baseline > $O/staged_blit.json 2> $O/staged_blit.err || exit $?
