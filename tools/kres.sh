#!/bin/bash
# Register / LDS / spill / occupancy remarks of the volume kernels (device-only compile, no GPU):
#   bash tools/kres.sh [kernel-name-regex]
cd "$(dirname "$0")/../parmmg_amd/csrc" || exit 1
hipcc --offload-arch=gfx950 -O3 -mllvm -amdgpu-sched-strategy=max-memory-clause -std=c++17 -ffp-contract=off -I../../include -c pmmg_hip.hip -o /tmp/kres.o \
  --offload-device-only -Rpass-analysis=kernel-resource-usage 2>&1 |
  grep -A11 -E "Function Name: .*${1:-k_vol}" | grep -E "Function Name|VGPRs: |Spill|Occupancy|LDS Size"
