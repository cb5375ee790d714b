#!/bin/bash
# Print VGPR/AGPR/SGPR/scratch/occupancy/LDS per kernel of a HIP source (gfx950), one line each,
# compiled with the same device flags as cs336_systems/_native/build.py.
# usage: scripts/kernel_resources.sh csrc/flash_attn/fa_fwd.hip [regex-filter]
src=$1; filt=${2:-.}
hipcc ${KR_FLAGS:-} -O3 -std=c++17 --offload-arch=gfx950 -mllvm -amdgpu-mfma-vgpr-form -Icsrc/include -Icsrc/flash_attn \
  -c "$src" -o /tmp/_kr.o -Rpass-analysis=kernel-resource-usage 2>&1 \
  | sed -n 's/.*remark: *//p' | sed 's/ \[-Rpass-analysis=kernel-resource-usage\]//' | awk '
  /Function Name:/ {if (line!="") print line; line=sprintf("%s", $3); next}
  /^ *VGPRs:/ {line=line" vgpr="$2} /^ *AGPRs:/ {line=line" agpr="$2} /TotalSGPRs/ {line=line" sgpr="$2}
  /ScratchSize/ {line=line" scratch="$NF} /Occupancy/ {line=line" occ="$NF} /LDS Size/ {line=line" lds="$NF}
  END {print line}' | c++filt | sed 's/(cs336::[A-Za-z]*Params)//' | grep -E "$filt"
