#!/bin/bash
# Round 5, GPU call v: resolve rework (delayed value stores, unrolled pointer
# jumping, per-thread Horner CRC) -- tests, then decode probe A/B against the
# previous decoder (decbase), resolve without the register cap (w1) and
# 8-record op bursts (e8).
set -uo pipefail
R=$PWD
O=$R/gpurun_out/r05v
mkdir -p $O
T() { timeout -k 10 "$@"; }
T 500 python -u -m pytest tests/test_gpu_lossy.py tests/test_gunzip.py -x -q --timeout 120 --timeout-method thread > $O/pytest_lossy.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest_lossy.log
[ $rc -eq 0 ] || exit 11
OFL_TLZ_DEC_STATS=1 T 300 python -u tools/kc_inflate_probe.py > $O/stats.txt 2> $O/stats.err || exit 12
for r in 1 2; do
  for v in main decbase w1 e8; do
    if [ $v = main ]; then L=$R/openfl_amd/lib/libofl_codec.so; else L=$R/tools/bin/var/libofl_$v.so; fi
    OFL_CODEC_LIB=$L T 300 python -u tools/kc_inflate_probe.py > $O/probe_${v}_$r.json 2> $O/probe_${v}_$r.err || exit 13
  done
done
echo "r05v done"
