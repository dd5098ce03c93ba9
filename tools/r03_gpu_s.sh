#!/bin/bash
# Round 3, GPU call S: gzip batches double-buffered with the pack (PCIe write
# into the mapped output) on a side stream (default) vs one stream (pack1,
# variant library of the previous tree): lossy + e2e GPU tests, KC pipeline
# alternated, kernel trace.  gpurun_out/r3s/.
set -uo pipefail
R=$PWD
O=$R/gpurun_out/r3s
mkdir -p $O
T() { timeout -k 10 "$@"; }
T 500 python -u -m pytest tests/test_gpu_lossy.py tests/test_gpu_e2e.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || exit 11
for rep in 1 2 3; do
  for v in base pack1; do
    if [ $v = base ]; then unset OFL_CODEC_LIB; else export OFL_CODEC_LIB=$R/openfl_amd/lib/variants/libofl_codec_$v.so; fi
    T 200 python -u tools/kc_bench.py --steps 10 --warmup 2 > $O/kc_${rep}_$v.json 2> $O/kc_${rep}_$v.err || exit 12
  done
done
