#!/bin/bash
# Round 3, GPU call U: ResNet-50 on the fused one-queue schedule, row passes
# with two blocks per CU (default below 4 tiles per CU) vs the persistent
# one-block kernels (OFL_EDEN_ROW2=0) vs also the one-block encode pass C
# (OFL_EDEN_ROWC2=0), alternated; a kernel trace of each.
set -uo pipefail
R=$PWD
O=$R/gpurun_out/r3u
mkdir -p $O
T() { timeout -k 10 "$@"; }
for rep in 1 2 3; do
  for v in "row2" "row1:OFL_EDEN_ROW2=0" "row1c1:OFL_EDEN_ROW2=0 OFL_EDEN_ROWC2=0"; do
    n=${v%%:*}; e=""; [ "$n" != "$v" ] && e=${v#*:}
    T 300 env $e python -u bench.py --workload uniform_1gib --steps 3 --warmup 1 --also resnet50_fp32 --also-steps 400 --no-cpu-baseline > $O/rn_${rep}_$n.json 2> $O/rn_${rep}_$n.err || exit 16
  done
done
cd /tmp && export TMPDIR=/tmp
T 300 env OFL_EDEN_ROW2=0 rocprofv3 --kernel-trace --output-format csv -d $O/trace_row1 -o k -- python3 $R/bench.py --workload resnet50_fp32 --steps 20 --warmup 5 --also "" --no-cpu-baseline --no-kernel-events > $O/trace_row1.json 2> $O/trace_row1.err || exit 18
