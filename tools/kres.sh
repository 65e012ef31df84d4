#!/bin/bash
# Per-kernel VGPR / AGPR / spill / occupancy of one HIP source (compile-only, gfx950):
#   bash tools/kres.sh loner_amd/csrc/hashgrid_bwd.hip [name-filter]
f=$1; pat=${2:-.}
extra=""; [ "$(basename $f)" = hashgrid_bwd.hip ] && extra="-fno-slp-vectorize"
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -ffp-contract=off $extra ${DEFS:-} -I $(dirname $0)/../include \
  -c $f -o /tmp/kres.o -Rpass-analysis=kernel-resource-usage 2>&1 \
  | grep -E "Function Name|VGPRs:|AGPRs:|VGPRs Spill|Occupancy|LDS Size" \
  | sed -E 's/.*remark: *//; s/ \[-Rpass.*//' | paste - - - - - - | grep -E "$pat" \
  | sed -E 's/Function Name: //' | awk -F'\t' '{printf "%-90s %s | %s | %s | %s | %s\n", substr($1,1,90), $2, $3, $4, $5, $6}'
