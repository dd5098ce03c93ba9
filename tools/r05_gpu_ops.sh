#!/bin/bash
# Round 5: ops lane loop: block-granular bound check, one branch for a copy's checks -- lossy tests, decode probe and KC A/B against the previous ops (ops0).
set -uo pipefail
R=$PWD
O=$R/gpurun_out/r05ops
mkdir -p $O
T() { timeout -k 10 "$@"; }
T 500 python -u -m pytest tests/test_gpu_lossy.py tests/test_gunzip.py -x -q --timeout 120 --timeout-method thread > $O/pytest_lossy.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest_lossy.log
[ $rc -eq 0 ] || exit 11
for r in 1 2; do
  OFL_TLZ_DEC_STATS=1 T 300 python -u tools/kc_inflate_probe.py > $O/stats_new_$r.txt 2> $O/stats_new_$r.err || exit 12
  OFL_CODEC_LIB=$R/tools/bin/var/libofl_ops0.so OFL_TLZ_DEC_STATS=1 T 300 python -u tools/kc_inflate_probe.py > $O/stats_old_$r.txt 2> $O/stats_old_$r.err || exit 13
done
for r in 1 2; do
  T 300 python -u tools/kc_bench.py --steps 10 --warmup 4 > $O/kc_new_$r.json 2> $O/kc_new_$r.err || exit 14
  OFL_CODEC_LIB=$R/tools/bin/var/libofl_ops0.so T 300 python -u tools/kc_bench.py --steps 10 --warmup 4 > $O/kc_old_$r.json 2> $O/kc_old_$r.err || exit 15
done
echo "r05ops done"
