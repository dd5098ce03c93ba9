#!/bin/bash
# Build libofl_codec.so from another revision's eden_kernels.hip (the other
# sources from the working tree) for kernel A/Bs with OFL_CODEC_LIB:
#   bash tools/build_variant.sh REV OUT.so [extra hipcc flags]
set -euo pipefail
REV=$1; OUT=$2; shift 2
R=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d)
cp "$R"/openfl_amd/csrc/*.hip "$R"/openfl_amd/csrc/*.h "$R"/openfl_amd/csrc/*.inc "$T"/
git -C "$R" show "$REV":openfl_amd/csrc/eden_kernels.hip > "$T"/eden_kernels.hip
mkdir -p "$(dirname "$OUT")"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -std=c++20 -O3 -fPIC -shared -Wno-unused-function "$@" \
    -I"$R"/include -I"$T" -o "$OUT" "$T"/eden_kernels.hip "$T"/lossy_kernels.hip "$T"/agg_kernels.hip \
    "$T"/deflate_kernels.hip -lz
rm -rf "$T"
