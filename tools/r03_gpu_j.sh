#!/bin/bash
# Round 3, GPU call J: is the batched loopback slower with the threaded seed
# sum?  tools/e2e_bench.py --modes batched, alternated with OFL_SUM_THREADS=1
# (the plain chain everywhere).  Outputs under gpurun_out/r3j/.
set -uo pipefail
R=$PWD
O=$R/gpurun_out/r3j
mkdir -p $O
T() { timeout -k 10 "$@"; }
for rep in 1 2 3; do
  T 200 python -u tools/e2e_bench.py --modes batched,plugin --out $O/e2e_mt_$rep.json > $O/e2e_mt_$rep.log 2>&1 || exit 11
  T 200 env OFL_SUM_THREADS=1 python -u tools/e2e_bench.py --modes batched,plugin --out $O/e2e_st_$rep.json > $O/e2e_st_$rep.log 2>&1 || exit 12
done
