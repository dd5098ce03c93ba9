#!/bin/bash
# Round 5, GPU call ac: bench.py with GPU_MAX_HW_QUEUES=8 (its default now)
# vs 4, and kc_bench with 3 streams made first at 8 queues.
set -uo pipefail
R=$PWD
O=$R/gpurun_out/r05ac
mkdir -p $O
T() { timeout -k 10 "$@"; }
T 600 python -u bench.py > $O/bench_q8.json 2> $O/bench_q8.err || exit 11
GPU_MAX_HW_QUEUES=4 T 600 python -u bench.py > $O/bench_q4.json 2> $O/bench_q4.err || exit 12
T 600 python -u bench.py > $O/bench_q8b.json 2> $O/bench_q8b.err || exit 13
for r in 1 2; do
  GPU_MAX_HW_QUEUES=8 T 300 python -u tools/kc_bench.py --steps 10 --warmup 4 --extra-streams 3 > $O/kc_q8_$r.json 2> $O/kc_q8_$r.err || exit 14
done
echo "r05ac done"
