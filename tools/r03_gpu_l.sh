#!/bin/bash
# Round 3, GPU call L: a ResNet-50 step's timeline (rocprofv3 --kernel-trace,
# per-dispatch start / end) for tools/resnet_timeline.py.  gpurun_out/r3l/.
set -uo pipefail
R=$PWD
O=$R/gpurun_out/r3l
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o k -- python3 $R/bench.py --workload resnet50_fp32 --steps 20 --warmup 5 --also '' --no-cpu-baseline --no-kernel-events > $O/bench.json 2> $O/trace.err || exit 11
