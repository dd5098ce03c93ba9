#!/bin/bash
# Round 5, GPU call g: pipelined inflate (H2D pieces inflated as they land)
# and 11 chain candidates: lossy GPU tests, KC line per piece count.
set -uo pipefail
R=$PWD
O=$R/gpurun_out/r05g
mkdir -p $O
T() { timeout -k 10 "$@"; }
T 400 python -u -m pytest tests/test_gpu_lossy.py -x -q --timeout 120 --timeout-method thread > $O/pytest_lossy.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest_lossy.log
[ $rc -eq 0 ] || exit 11
for p in 4 1 2 6 4; do
  OFL_INFLATE_PIECES=$p T 300 python -u tools/kc_bench.py --steps 10 --warmup 2 > $O/kc_p$p.json 2> $O/kc_p$p.err || exit 15
  python -c "import json;d=json.load(open('$O/kc_p$p.json'));print('pieces=$p',d['value'],d['ms_per_step'],d['phases_ms'],d['wire_ratio'])" >> $O/summary.txt
done
echo "r05g done"
