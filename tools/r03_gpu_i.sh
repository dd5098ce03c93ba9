#!/bin/bash
# Round 3, GPU call I: float4 ws tile I/O in k_enc_rowA / k_dec_rowC (layout
# L3F) -- the -m gpu suite (bit-identity to the other schedules and the
# oracle), then an alternated Llama-step A/B against the dword L3 build
# (OFL_ROW_WS4=0); the seed-sum phase timings on the box.  gpurun_out/r3i/.
set -uo pipefail
R=$PWD
O=$R/gpurun_out/r3i
mkdir -p $O
T() { timeout -k 10 "$@"; }
T 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest_gpu.log
[ $rc -eq 0 ] || exit 13
i=0
for v in base ws1 base ws1 base ws1; do
  i=$((i+1))
  if [ $v = base ]; then unset OFL_CODEC_LIB; else export OFL_CODEC_LIB=$R/openfl_amd/lib/variants/libofl_codec_$v.so; fi
  T 240 python -u bench.py --steps 10 --warmup 3 --also '' --no-cpu-baseline > $O/ab_${i}_$v.json 2> $O/ab_${i}_$v.err || exit 14
done
unset OFL_CODEC_LIB
OFL_SUM_DEBUG=1 T 120 python -u tools/sum_rate.py > $O/sum_rate.log 2>&1 || exit 15
