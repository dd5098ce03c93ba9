#!/bin/bash
# Round 5, GPU call af: bench.py default (HIP's 4 HW queues) x2 with the
# high-priority gzip DMA stream and the shared inflate side streams.
set -uo pipefail
R=$PWD
O=$R/gpurun_out/r05af
mkdir -p $O
T() { timeout -k 10 "$@"; }
T 600 python -u bench.py > $O/bench_1.json 2> $O/bench_1.err || exit 12
T 600 python -u bench.py > $O/bench_2.json 2> $O/bench_2.err || exit 13
echo "r05af done"
