#!/bin/bash
# Round 5, GPU call p: KC decode timeline and piece / side-stream sweep (tools/kc_inflate_probe.py).
set -uo pipefail
R=$PWD
O=$R/gpurun_out/r05p
mkdir -p $O
T() { timeout -k 10 "$@"; }
T 300 python -u tools/kc_inflate_probe.py > $O/probe2.json 2> $O/probe2.err || exit 11
echo "r05p done"
