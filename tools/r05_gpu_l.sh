#!/bin/bash
# Round 5, GPU call l: the fused-LUT inflate: lossy GPU tests, KC line.
set -uo pipefail
R=$PWD
O=$R/gpurun_out/r05l
mkdir -p $O
T() { timeout -k 10 "$@"; }
T 400 python -u -m pytest tests/test_gpu_lossy.py -x -q --timeout 120 --timeout-method thread > $O/pytest_lossy.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest_lossy.log
[ $rc -eq 0 ] || exit 11
for r in 1 2 3; do
  T 300 python -u tools/kc_bench.py --steps 15 --warmup 3 > $O/kc_$r.json 2> $O/kc_$r.err || exit 15
  python -c "import json;d=json.load(open('$O/kc_$r.json'));print(d['value'],d['ms_per_step'],d['phases_ms'],d['wire_ratio'])" >> $O/summary.txt
done
echo "r05l done"
