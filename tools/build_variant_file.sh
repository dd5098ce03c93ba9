#!/bin/bash
# Build libofl_codec.so with one source file taken from another revision (the
# other sources from the working tree), for kernel A/Bs with OFL_CODEC_LIB:
#   bash tools/build_variant_file.sh REV FILE OUT.so [extra hipcc flags]
# FILE: a name under openfl_amd/csrc/, e.g. deflate_kernels.hip
set -euo pipefail
REV=$1; FILE=$2; OUT=$3; shift 3
R=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d)
cp "$R"/openfl_amd/csrc/*.hip "$R"/openfl_amd/csrc/*.cpp "$R"/openfl_amd/csrc/*.h "$R"/openfl_amd/csrc/*.inc "$T"/
git -C "$R" show "$REV":openfl_amd/csrc/"$FILE" > "$T"/"$FILE"
mkdir -p "$(dirname "$OUT")"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -std=c++20 -O3 -fPIC -shared -Wno-unused-function "$@" \
    -I"$R"/include -I"$T" -o "$OUT" "$T"/eden_kernels.hip "$T"/lossy_kernels.hip "$T"/agg_kernels.hip \
    "$T"/deflate_kernels.hip "$T"/serial_sum.cpp -lz
rm -rf "$T"
