#!/bin/bash
# Register / LDS / scratch use of the kernels in a hipcc-built object (gfx950), from the
# code object's AMDGPU metadata: tools/co_resources.sh reed-solomon-cc_amd/build/rs_lowlds.o [name-regex]
set -e
T=$(mktemp -d)
/opt/rocm/lib/llvm/bin/llvm-objcopy --dump-section=.hip_fatbin=$T/fat.bin "$1"
/opt/rocm/lib/llvm/bin/clang-offload-bundler --unbundle --type=o --input=$T/fat.bin \
  --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output=$T/k.co
/opt/rocm/lib/llvm/bin/llvm-readelf --notes $T/k.co | awk -v pat="${2:-.}" '
  /^ *- \.agpr_count|^ *- \.args/ {if (name != "" && name ~ pat) print name, out; name=""; out=""}
  /\.name:/ {name=$2}
  /\.(vgpr_count|sgpr_count|vgpr_spill_count|sgpr_spill_count|private_segment_fixed_size|group_segment_fixed_size):/ {out=out" "$1$2}
  END {if (name != "" && name ~ pat) print name, out}'
rm -rf $T
