#!/bin/bash
# Round 5, GPU call e: the KC line after the batch-copy reorder; A/B streams.
set -uo pipefail
R=$PWD
O=$R/gpurun_out/r05e
mkdir -p $O
T() { timeout -k 10 "$@"; }
T 400 python -u -m pytest tests/test_gpu_lossy.py -x -q --timeout 120 --timeout-method thread > $O/pytest_lossy.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest_lossy.log
[ $rc -eq 0 ] || exit 11
T 200 python -u tools/tlz_ab.py new > $O/ab.jsonl 2> $O/ab_new.err || exit 13
T 300 python -u tools/kc_bench.py --steps 10 --warmup 2 > $O/kc_new.json 2> $O/kc_new.err || exit 15
OFL_GZ_FILL_TRACE=1 T 200 python -u tools/kc_bench.py --steps 3 --warmup 1 > $O/kc_trace.json 2> $O/kc_fill_trace.txt || exit 17
echo "r05e done"
