#!/bin/bash
# Round 3, GPU call A: stream calibration in the codec's shapes, the -m gpu
# suite, and an nt cache-policy A/B of the large-slice passes (library
# variants built by tools/build_flags_variant.sh), then the default bench.
set -uo pipefail
O=gpurun_out/r3a
mkdir -p $O
T() { timeout -k 10 "$@"; }
T 120 ./tools/bin/streambench3 > $O/streambench3.txt 2>&1 || exit 11
T 120 ./tools/bin/streambench > $O/streambench1_fixed_bpe.txt 2>&1 || exit 12
T 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 13
i=0
for v in base ld2 st2 both2 base ld2 both2 base; do
  i=$((i+1))
  if [ $v = base ]; then unset OFL_CODEC_LIB; else export OFL_CODEC_LIB=$PWD/openfl_amd/lib/variants/libofl_codec_$v.so; fi
  T 240 python -u bench.py --steps 10 --warmup 3 --also '' --no-cpu-baseline > $O/ab_${i}_$v.json 2> $O/ab_${i}_$v.err || exit 14
done
unset OFL_CODEC_LIB
T 400 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err || exit 15
T 200 python -u tools/kc_bench.py --steps 10 --warmup 2 > $O/kc_bench.json 2> $O/kc_bench.err || exit 16
