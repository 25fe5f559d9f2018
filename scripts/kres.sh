#!/bin/bash
# Register / LDS / spill metadata of the kernels in libmipx.so whose name matches $1
# (llvm-readobj notes of the extracted gfx950 code objects)
set -eu
LIB=${LIB:-$(cd "$(dirname "$0")/.." && pwd)/imaginary_amd/libmipx.so}
T=$(mktemp -d); trap 'rm -rf "$T"' EXIT
cp "$LIB" "$T/lib.so"; (cd "$T" && /opt/rocm/lib/llvm/bin/llvm-objdump --offloading lib.so > /dev/null)
for f in "$T"/*gfx950*; do
  /opt/rocm/lib/llvm/bin/llvm-readobj --notes "$f" | grep -E "\.name:|\.vgpr_count|\.sgpr_count|group_segment_fixed_size|spill_count" \
    | paste - - - - - - | sed 's/  */ /g'
done | c++filt | grep -E "${1:-.}"
