#!/bin/bash
# Round 3, GPU call P: height-6 middle passes inside the fused column +
# small-set launch (col_body<6>, default) vs their own k_col6<6> launch
# (OFL_EDEN_COLM6=0): -m gpu suite, ResNet-50 alternated, Llama control.
set -uo pipefail
R=$PWD
O=$R/gpurun_out/r3p
mkdir -p $O
T() { timeout -k 10 "$@"; }
T 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest_gpu.log
[ $rc -eq 0 ] || exit 13
for rep in 1 2 3; do
  for v in "colm6" "sep6:OFL_EDEN_COLM6=0"; do
    n=${v%%:*}; e=""; [ "$n" != "$v" ] && e=${v#*:}
    T 300 env $e python -u bench.py --workload uniform_1gib --steps 3 --warmup 1 --also resnet50_fp32 --also-steps 400 --no-cpu-baseline > $O/rn_${rep}_$n.json 2> $O/rn_${rep}_$n.err || exit 16
  done
done
T 300 python -u bench.py --steps 10 --warmup 3 --also '' --no-cpu-baseline > $O/llama.json 2> $O/llama.err || exit 17
