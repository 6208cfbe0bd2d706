#!/bin/bash
# Per-kernel VGPR / SGPR / occupancy / LDS of one csrc file, one line per kernel:
#   bash profiles/tools/resources.sh tsdf_kernels.hip [name-regex] [extra hipcc flags...]
cd "$(dirname "$0")/../../noetic-slam_amd/csrc" || exit 1
f=$1; pat=${2:-.}; shift 2 2>/dev/null
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off \
  -fhip-fp32-correctly-rounded-divide-sqrt -fno-gpu-flush-denormals-to-zero "$@" \
  -c -o /dev/null "$f" -Rpass-analysis=kernel-resource-usage 2>&1 | awk -v pat="$pat" '
  /Function Name:/ { if (name != "" && name ~ pat) print name, v, s, o, l; name=$NF; sub(/\[.*/, "", name); n=split($0, a, "Function Name: "); split(a[2], b, " "); name=b[1]; v=s=o=l="" }
  /VGPRs:/ && !/AGPR/ { v="vgpr=" $(NF-1) }
  /TotalSGPRs:/ { s="sgpr=" $(NF-1) }
  /Occupancy/ { o="occ=" $(NF-1) }
  /LDS Size/ { l="lds=" $(NF-1) }
  /error/ { print }
  END { if (name != "" && name ~ pat) print name, v, s, o, l }'
