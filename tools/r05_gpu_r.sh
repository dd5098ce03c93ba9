#!/bin/bash
# Round 5, GPU call r: kernel trace of the KC decode probe (ops / resolve durations).
set -uo pipefail
R=$PWD
O=$R/gpurun_out/r05r
mkdir -p $O
T() { timeout -k 10 "$@"; }
cd /tmp && export TMPDIR=/tmp
T 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o k -- python3 $R/tools/kc_inflate_probe.py > $O/probe.json 2> $O/probe.err || exit 11
echo "r05r done"
