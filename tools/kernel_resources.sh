#!/bin/bash
# Per-kernel VGPR/AGPR/SGPR/LDS/scratch of the gfx950 code objects (offline, no GPU).
# Usage: bash tools/kernel_resources.sh [file.hip ...]
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
C=$R/pino-locoman_amd/csrc
T=$(mktemp -d)
for f in ${@:-k_admm k_factor k_eval k_qp}; do
  /opt/rocm/bin/hipcc -std=c++17 -O3 --offload-arch=gfx950 --cuda-device-only -c -I "$C" -I "$R/include" \
    "$C/${f%.hip}.hip" -o "$T/$f.bundle" 2>/dev/null
  /opt/rocm/lib/llvm/bin/clang-offload-bundler --unbundle --type=o --input="$T/$f.bundle" \
    --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output="$T/$f.co"
  /opt/rocm/lib/llvm/bin/llvm-readelf --notes "$T/$f.co" | grep -E "^ +\.name:|\.vgpr_count|\.agpr_count|\.sgpr_count|group_segment_fixed|\.vgpr_spill|private_segment_fixed" \
    | awk '/\.name:/{if(n!="")print n, s; n=$2; s=""; next}{s=s" "$1$2}END{print n, s}'
done
rm -rf "$T"
