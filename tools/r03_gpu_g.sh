#!/bin/bash
# Round 3, GPU call G: where the ResNet-50 small-set launch should run --
# beside the wave on the side stream (default), first on the caller's stream
# (OFL_EDEN_SMALLSTREAM=0), or with no side stream at all (--streams 1);
# eager and graph, alternated; then a kernel trace of the one-stream variant.
set -uo pipefail
R=$PWD
O=$R/gpurun_out/r3g
mkdir -p $O
T() { timeout -k 10 "$@"; }
for rep in 1 2; do
  for v in "default" "callerfirst:OFL_EDEN_SMALLSTREAM=0" "onestream:OFL_EDEN_SMALLSTREAM=0:1"; do
    n=${v%%:*}; rest=${v#*:}; e=""; st=""
    [ "$n" != "$v" ] && e=${rest%%:*} && [ "$rest" != "$e" ] && st="--streams ${rest#*:}"
    T 300 env $e python -u bench.py --workload uniform_1gib --steps 3 --warmup 1 --also resnet50_fp32 --also-steps 400 --no-cpu-baseline $st > $O/rn_${rep}_$n.json 2> $O/rn_${rep}_$n.err || exit 16
  done
done
cd /tmp && export TMPDIR=/tmp
T 300 env OFL_EDEN_SMALLSTREAM=0 rocprofv3 --kernel-trace --stats --output-format csv -d $O/rn_trace1 -o k -- python3 $R/bench.py --workload resnet50_fp32 --steps 30 --warmup 5 --also '' --no-cpu-baseline --no-kernel-events --streams 1 > $O/rn_trace1.json 2> $O/rn_trace1.err || exit 21
