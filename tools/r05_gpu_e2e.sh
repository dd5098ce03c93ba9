#!/bin/bash
# Round 5: end-to-end ResNet-50 loopback repeats (batched path variance), unbound and NUMA-bound.
set -uo pipefail
R=$PWD
O=$R/gpurun_out/r05e2e
mkdir -p $O
T() { timeout -k 10 "$@"; }
for r in 1 2; do
  T 300 python -u tools/e2e_bench.py --modes plugin,batched --out $O/e2e_free_$r.json > $O/e2e_free_$r.log 2>&1 || exit 11
  T 300 python -u tools/e2e_bench.py --modes plugin,batched --numa-bind --out $O/e2e_bind_$r.json > $O/e2e_bind_$r.log 2>&1 || exit 12
done
echo "r05e2e done"
