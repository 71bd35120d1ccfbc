#!/bin/bash
set -o pipefail
bash tools/quick32.sh
grep -h "fused vs unfused" gpurun_out/quick32/tests.log || true
