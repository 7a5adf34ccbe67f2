#!/bin/bash
# kernel resource usage (VGPRs, spills, LDS, occupancy) of the HIP library's kernels: tools/kres.sh [SRC_DIR] [flags]
src=${1:-nascargymnasium_amd/csrc}; shift
hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -fno-fast-math -fPIC -std=c++17 -Wno-unused-value -Wno-unused-result \
  --cuda-device-only -c -o /tmp/kres.o -Rpass-analysis=kernel-resource-usage "$@" "$src/nascar_kernels.hip" 2>&1 \
  | grep -E "Function Name|VGPRs:|AGPRs|ScratchSize|Occupancy|LDS Size" | sed 's/.*remark: //' | paste - - - - - - | grep -E "model_kernel|logic_kernel|ray_sensor|rollout_kernel"
