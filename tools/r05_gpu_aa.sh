#!/bin/bash
# Round 5, GPU call aa: KC pipeline after N other streams exist (HW queue sharing?), alternated.
set -uo pipefail
R=$PWD
O=$R/gpurun_out/r05aa
mkdir -p $O
T() { timeout -k 10 "$@"; }
for r in 1 2; do
  for n in 0 3 6; do
    T 300 python -u tools/kc_bench.py --steps 10 --warmup 4 --extra-streams $n > $O/kc_s${n}_$r.json 2> $O/kc_s${n}_$r.err || exit 11
  done
done
echo "r05aa done"
