#!/bin/bash
# Per-kernel VGPR / scratch / occupancy of a HIP source (hipcc -Rpass-analysis).
f=$1
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -I"$(dirname "$0")/../include" \
  -I"$(dirname "$0")/../visionx-slam_amd/csrc" -x hip -c "$f" -o /tmp/kres.o -Rpass-analysis=kernel-resource-usage 2>&1 |
  grep -E "Function Name|VGPRs:|ScratchSize|Occupancy" | sed -E 's/.*remark: +//; s/ \[-Rpass.*//' | paste - - - - |
  sed -E 's/Function Name: _ZN2vx12_GLOBAL__N_1[0-9]+//'
