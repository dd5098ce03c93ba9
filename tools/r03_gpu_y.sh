#!/bin/bash
# Round 3, GPU call Y: device inflate residency -- __launch_bounds__(64, 8)
# (SGPRs capped at 78, 8 waves per SIMD) with / without an 8-bit literal
# table (LDS for 32 members per CU) vs the default (106 SGPRs, 7 waves):
# the lossy GPU tests on the lit8w8 variant, the KC pipeline alternated, the
# inflate kernel's rocprof stats per variant.  gpurun_out/r3y/.
set -uo pipefail
R=$PWD
O=$R/gpurun_out/r3y
mkdir -p $O
T() { timeout -k 10 "$@"; }
V=$R/openfl_amd/lib/variants
OFL_CODEC_LIB=$V/libofl_codec_lit8w8.so T 500 python -u -m pytest tests/test_gpu_lossy.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_lit8w8.log 2>&1 || exit 11
for rep in 1 2 3; do
  for v in base lit8w8 w8 lit8; do
    if [ $v = base ]; then unset OFL_CODEC_LIB; else export OFL_CODEC_LIB=$V/libofl_codec_$v.so; fi
    T 200 python -u tools/kc_bench.py --steps 10 --warmup 2 > $O/kc_${rep}_$v.json 2> $O/kc_${rep}_$v.err || exit 12
  done
done
unset OFL_CODEC_LIB
cd /tmp && export TMPDIR=/tmp
for v in base lit8w8 w8; do
  if [ $v = base ]; then L=""; else L="OFL_CODEC_LIB=$V/libofl_codec_$v.so"; fi
  T 300 env $L rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$v -o k -- python3 $R/tools/kc_bench.py --steps 3 --warmup 1 > $O/trace_$v.log 2>&1 || exit 13
done
