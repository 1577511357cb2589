#!/bin/bash
# VGPR / AGPR / scratch / LDS of every kernel in a built object (code-object metadata).
# usage: scripts/kernel_resources.sh pde-engine_amd/lib/obj/pdeval_grid.o [name-filter]
set -e
B=/opt/rocm/lib/llvm/bin
T=$(mktemp -d)
$B/llvm-objcopy --dump-section=.hip_fatbin=$T/fb.bin "$1" $T/copy.o
$B/clang-offload-bundler --unbundle --type=o --input=$T/fb.bin --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output=$T/co
$B/llvm-readelf --notes $T/co | grep -E "^\s+(- )?\.(name|private_segment_fixed_size|vgpr_count|agpr_count|group_segment_fixed_size):" |
  awk '/\.agpr_count/{a=$NF} /group_segment_fixed_size/{l=$NF} /\.name:/{n=$NF} /private_segment_fixed_size/{p=$NF} /\.vgpr_count/{print n, "vgpr", $NF, "agpr", a, "scratch", p, "lds", l}' |
  grep -E "${2:-.}" | c++filt -t 2>/dev/null || true
rm -rf $T
