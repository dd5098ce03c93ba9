#!/bin/bash
# Round 5, GPU call ad: library side streams shared (ofl_side_stream) --
# lossy + parity GPU tests, bench.py default x2, kc_bench with 3 streams made
# first at 4 HW queues x2.
set -uo pipefail
R=$PWD
O=$R/gpurun_out/r05ad
mkdir -p $O
T() { timeout -k 10 "$@"; }
T 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest_gpu.log
[ $rc -eq 0 ] || exit 11
T 600 python -u bench.py > $O/bench_1.json 2> $O/bench_1.err || exit 12
T 600 python -u bench.py > $O/bench_2.json 2> $O/bench_2.err || exit 13
for r in 1 2; do
  GPU_MAX_HW_QUEUES=4 T 300 python -u tools/kc_bench.py --steps 10 --warmup 4 --extra-streams 3 > $O/kc_q4s3_$r.json 2> $O/kc_q4s3_$r.err || exit 14
done
echo "r05ad done"
