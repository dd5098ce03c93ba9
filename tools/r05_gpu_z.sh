#!/bin/bash
# Round 5, GPU call z: KC pipeline with the process bound to the GPU's NUMA
# node (openfl_amd.numa) vs unbound, alternated; then the default bench line.
set -uo pipefail
R=$PWD
O=$R/gpurun_out/r05z
mkdir -p $O
T() { timeout -k 10 "$@"; }
for r in 1 2 3; do
  T 300 python -u tools/kc_bench.py --steps 10 --warmup 4 > $O/kc_bind_$r.json 2> $O/kc_bind_$r.err || exit 11
  T 300 python -u tools/kc_bench.py --steps 10 --warmup 4 --no-numa-bind > $O/kc_free_$r.json 2> $O/kc_free_$r.err || exit 12
done
T 600 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err || exit 13
echo "r05z done"
