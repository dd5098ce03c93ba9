#!/bin/bash
# Round 5, GPU call w: the KC leg inside bench.py vs alone -- default bench
# (all legs), bench with only the KC leg, then the standalone KC bench.
set -uo pipefail
R=$PWD
O=$R/gpurun_out/r05w
mkdir -p $O
T() { timeout -k 10 "$@"; }
T 600 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err || exit 11
T 400 python -u bench.py --also kc_uniform_1gib --no-cpu-baseline > $O/bench_kconly.json 2> $O/bench_kconly.err || exit 12
T 300 python -u tools/kc_bench.py --steps 10 --warmup 4 > $O/kc_bench.json 2> $O/kc_bench.err || exit 13
echo "r05w done"
