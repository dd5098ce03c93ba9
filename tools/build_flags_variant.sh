#!/bin/bash
# Build libofl_codec.so from the WORKING TREE with extra hipcc flags (tuning
# constants such as -DOFL_LD_AUX=2) for A/Bs with OFL_CODEC_LIB:
#   bash tools/build_flags_variant.sh OUT.so [extra hipcc flags]
set -euo pipefail
OUT=$1; shift
R=$(cd "$(dirname "$0")/.." && pwd)
C=$R/openfl_amd/csrc
mkdir -p "$(dirname "$OUT")"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -std=c++20 -O3 -fPIC -shared -Wno-unused-function "$@" \
    -I"$R"/include -I"$C" -o "$OUT" "$C"/eden_kernels.hip "$C"/lossy_kernels.hip "$C"/agg_kernels.hip \
    "$C"/deflate_kernels.hip "$C"/serial_sum.cpp -lz
