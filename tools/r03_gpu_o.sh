#!/bin/bash
# Round 3, GPU call O: the small-set groups fused into the one-wave plan's
# k_col_multi launch (k_*_colm_set, no side stream, default) vs the small-set
# launch beside the wave on the side stream (OFL_EDEN_FUSESET=0): the -m gpu
# suite, ResNet-50 alternated (eager + graph), and the fused step's timeline.
set -uo pipefail
R=$PWD
O=$R/gpurun_out/r3o
mkdir -p $O
T() { timeout -k 10 "$@"; }
T 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest_gpu.log
[ $rc -eq 0 ] || exit 13
for rep in 1 2 3; do
  for v in "fused" "side:OFL_EDEN_FUSESET=0"; do
    n=${v%%:*}; e=""; [ "$n" != "$v" ] && e=${v#*:}
    T 300 env $e python -u bench.py --workload uniform_1gib --steps 3 --warmup 1 --also resnet50_fp32 --also-steps 400 --no-cpu-baseline > $O/rn_${rep}_$n.json 2> $O/rn_${rep}_$n.err || exit 16
  done
done
cd /tmp && export TMPDIR=/tmp
T 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o k -- python3 $R/bench.py --workload resnet50_fp32 --steps 20 --warmup 5 --also '' --no-cpu-baseline --no-kernel-events > $O/trace.json 2> $O/trace.err || exit 17
