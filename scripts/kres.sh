#!/bin/bash
# Per-kernel register / LDS / scratch report of the built objects (gfx950).
B=/opt/rocm/lib/llvm/bin
T=$(mktemp -d)
for o in "$@"; do
  $B/llvm-objcopy --dump-section=.hip_fatbin=$T/fb.bin "$o" 2>/dev/null || continue
  $B/clang-offload-bundler --unbundle --type=o --input=$T/fb.bin --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output=$T/k.co || continue
  echo "== $(basename $o)"
  $B/llvm-readelf --notes $T/k.co | grep -E "^\s+\.name:|\.vgpr_count|\.agpr_count|\.sgpr_count|private_segment_fixed_size|group_segment_fixed_size|vgpr_spill|sgpr_spill" | sed 's/^ *//' | awk '/^\.name:/{if(l)print l; l=$2; next}{l=l" "$0}END{print l}' | sed 's/\.\(group_segment_fixed_size\)/lds/;s/\.private_segment_fixed_size/scratch/' 
done
rm -rf $T
