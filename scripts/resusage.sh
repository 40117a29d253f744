#!/bin/bash
# Per-kernel VGPR / SGPR / occupancy / LDS of one HIP TU (gfx950).
#   scripts/resusage.sh re_amd/csrc/hip/ctr10.hip [filter]
cd "$(dirname "$0")/../re_amd" || exit 1
src=$(realpath --relative-to=. "../$1" 2>/dev/null || echo "$1")
/opt/rocm/bin/hipcc -O3 -fPIC -std=c++17 --offload-arch=gfx950 -I../include -Icsrc \
  -c "$src" -o /tmp/resusage.o -Rpass-analysis=kernel-resource-usage 2>&1 |
  grep -E "Function Name|VGPRs:|Occupancy|LDS Size|ScratchSize|VGPRs Spill" |
  sed -E 's/.*remark: *//; s/ \[-Rpass.*//' |
  paste - - - - - - | c++filt | grep -E "${2:-.}"
