#!/bin/bash
# Round 3, GPU call Q: device inflate with an 8-bit distance table (default)
# vs the 9-bit one (variant library built from the previous tree): the lossy
# GPU tests (gzip.decompress exactness), KC pipeline alternated, and the
# inflate kernel's rocprof stats.  gpurun_out/r3q/.
set -uo pipefail
R=$PWD
O=$R/gpurun_out/r3q
mkdir -p $O
T() { timeout -k 10 "$@"; }
T 500 python -u -m pytest tests/test_gpu_lossy.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || exit 11
for rep in 1 2 3; do
  for v in base inf9; do
    if [ $v = base ]; then unset OFL_CODEC_LIB; else export OFL_CODEC_LIB=$R/openfl_amd/lib/variants/libofl_codec_$v.so; fi
    T 200 python -u tools/kc_bench.py --steps 10 --warmup 2 > $O/kc_${rep}_$v.json 2> $O/kc_${rep}_$v.err || exit 12
  done
done
unset OFL_CODEC_LIB
cd /tmp && export TMPDIR=/tmp
T 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kc_trace -o k -- python3 $R/tools/kc_bench.py --steps 3 --warmup 1 > $O/kc_trace.log 2>&1 || exit 13
