#!/usr/bin/env bash
# Per-kernel register / spill / scratch usage of the render kernels (device compile only).
# usage: tools/resource_usage.sh [extra hipcc flags...]
set -eu
cd "$(dirname "$0")/.."
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off --cuda-device-only -c \
  -Rpass-analysis=kernel-resource-usage "$@" -o /tmp/myrt_ru.o myraytracer_amd/csrc/render.hip 2>&1 |
  sed -n 's/.*remark: *//p' | sed 's/ \[-Rpass-analysis=kernel-resource-usage\]//' |
  awk '/^Function Name: /{show=($3 ~ /render_kernel|render_full/); if (show) print $3; next}
       show && /^(TotalSGPRs|VGPRs|ScratchSize|Occupancy|SGPRs Spill|VGPRs Spill)/{printf "    %s\n", $0}'
