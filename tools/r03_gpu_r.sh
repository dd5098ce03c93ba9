#!/bin/bash
# Round 3, GPU call R: dword-store gzip pack kernel -- lossy GPU tests
# (gzip.decompress exactness), KC pipeline x3, kernel stats.  gpurun_out/r3r/.
set -uo pipefail
R=$PWD
O=$R/gpurun_out/r3r
mkdir -p $O
T() { timeout -k 10 "$@"; }
T 500 python -u -m pytest tests/test_gpu_lossy.py tests/test_gpu_e2e.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || exit 11
for rep in 1 2 3; do
  T 200 python -u tools/kc_bench.py --steps 10 --warmup 2 > $O/kc_$rep.json 2> $O/kc_$rep.err || exit 12
done
cd /tmp && export TMPDIR=/tmp
T 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kc_trace -o k -- python3 $R/tools/kc_bench.py --steps 3 --warmup 1 > $O/kc_trace.log 2>&1 || exit 13
