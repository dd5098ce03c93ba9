#!/bin/bash
# Round 5, GPU call s: ops one symbol per iteration + resolve prefetch -- tests, probe, KC x2.
# segment ahead -- lossy GPU tests, decode probe, KC line x2.
set -uo pipefail
R=$PWD
O=$R/gpurun_out/r05q
mkdir -p $O
T() { timeout -k 10 "$@"; }
T 500 python -u -m pytest tests/test_gpu_lossy.py tests/test_gunzip.py -x -q --timeout 120 --timeout-method thread > $O/pytest_lossy.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest_lossy.log
[ $rc -eq 0 ] || exit 11
T 300 python -u tools/kc_inflate_probe.py > $O/probe.json 2> $O/probe.err || exit 12
for r in 1 2; do
  T 300 python -u tools/kc_bench.py --steps 15 --warmup 3 > $O/kc_$r.json 2> $O/kc_$r.err || exit 15
  python -c "import json;d=json.load(open('$O/kc_$r.json'));print(d['value'],d['ms_per_step'],d['phases_ms'],d['wire_ratio'])" >> $O/summary.txt
done
echo "r05q done"
