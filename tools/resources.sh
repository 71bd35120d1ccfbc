#!/bin/bash
# Per-kernel VGPR / AGPR / spill / LDS usage of the gfx950 build (compiler remarks).
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared --cuda-device-only -c \
  -Rpass-analysis=kernel-resource-usage -o /tmp/res.o impala_amd/csrc/impala.hip 2>&1 |
  grep -E "Function Name|VGPRs:|AGPRs|ScratchSize|LDS Size|Occupancy" |
  sed -E 's/.*remark: //' | paste - - - - - - | sed -E 's/\s+/ /g' | cut -c1-400
