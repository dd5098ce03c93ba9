#!/bin/bash
# Round 3, GPU call M: height-6 middle passes inside k_col_multi (col_body<6>,
# default) vs their own k_col6<6> launch (OFL_EDEN_COLM6=0): the -m gpu suite,
# then ResNet-50 (and the 1 GiB set / Llama step as controls) alternated,
# eager and graph.  gpurun_out/r3m/.
set -uo pipefail
R=$PWD
O=$R/gpurun_out/r3m
mkdir -p $O
T() { timeout -k 10 "$@"; }
T 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest_gpu.log
[ $rc -eq 0 ] || exit 13
for rep in 1 2 3; do
  for v in "colm6" "sep6:OFL_EDEN_COLM6=0"; do
    n=${v%%:*}; e=""; [ "$n" != "$v" ] && e=${v#*:}
    T 300 env $e python -u bench.py --workload resnet50_fp32 --steps 400 --warmup 30 --also '' --no-cpu-baseline > $O/rn_${rep}_$n.json 2> $O/rn_${rep}_$n.err || exit 16
  done
done
for v in "colm6" "sep6:OFL_EDEN_COLM6=0"; do
  n=${v%%:*}; e=""; [ "$n" != "$v" ] && e=${v#*:}
  T 300 env $e python -u bench.py --steps 10 --warmup 3 --also uniform_1gib --no-cpu-baseline > $O/llama_$n.json 2> $O/llama_$n.err || exit 17
done
