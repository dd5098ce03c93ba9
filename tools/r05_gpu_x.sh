#!/bin/bash
# Round 5, GPU call x: does a large resident device allocation (the Llama
# leg's ~80 GB) slow the KC pipeline?  kc_bench alone vs with ballast.
set -uo pipefail
R=$PWD
O=$R/gpurun_out/r05x
mkdir -p $O
T() { timeout -k 10 "$@"; }
for r in 1 2; do
  for b in 0 80; do
    T 300 python -u tools/kc_bench.py --steps 10 --warmup 4 --ballast-gib $b > $O/kc_b${b}_$r.json 2> $O/kc_b${b}_$r.err || exit 11
  done
done
echo "r05x done"
