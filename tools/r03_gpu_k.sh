#!/bin/bash
# Round 3, GPU call K: k_dec_rowA with one more LDS exchange (L3 -> L3F) and
# float4 ws stores (-DOFL_DECA_WS4=1) vs default, Llama step alternated; the
# variant's bit-identity via the row2 / schedule tests.  gpurun_out/r3k/.
set -uo pipefail
R=$PWD
O=$R/gpurun_out/r3k
mkdir -p $O
T() { timeout -k 10 "$@"; }
OFL_CODEC_LIB=$R/openfl_amd/lib/variants/libofl_codec_deca4.so T 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "bit_identical or five_pass or decode" > $O/pytest_variant.log 2>&1 || exit 13
i=0
for v in base deca4 base deca4 base deca4; do
  i=$((i+1))
  if [ $v = base ]; then unset OFL_CODEC_LIB; else export OFL_CODEC_LIB=$R/openfl_amd/lib/variants/libofl_codec_$v.so; fi
  T 240 python -u bench.py --steps 10 --warmup 3 --also '' --no-cpu-baseline > $O/ab_${i}_$v.json 2> $O/ab_${i}_$v.err || exit 14
done
