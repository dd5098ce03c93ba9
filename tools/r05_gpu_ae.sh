#!/bin/bash
# Round 5, GPU call ae: gzip DMA on a high-priority stream, inflate pieces on
# the shared side streams -- bench.py default x2, kc_bench at 8 and at 4 HW
# queues with 3 streams made first.
set -uo pipefail
R=$PWD
O=$R/gpurun_out/r05ae
mkdir -p $O
T() { timeout -k 10 "$@"; }
T 300 python -u -m pytest tests/test_gpu_lossy.py -x -q --timeout 120 --timeout-method thread > $O/pytest_lossy.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest_lossy.log
[ $rc -eq 0 ] || exit 11
T 600 python -u bench.py > $O/bench_1.json 2> $O/bench_1.err || exit 12
T 600 python -u bench.py > $O/bench_2.json 2> $O/bench_2.err || exit 13
for r in 1 2; do
  T 300 python -u tools/kc_bench.py --steps 10 --warmup 4 > $O/kc_q8_$r.json 2> $O/kc_q8_$r.err || exit 14
  GPU_MAX_HW_QUEUES=4 T 300 python -u tools/kc_bench.py --steps 10 --warmup 4 --extra-streams 3 > $O/kc_q4s3_$r.json 2> $O/kc_q4s3_$r.err || exit 15
done
echo "r05ae done"
