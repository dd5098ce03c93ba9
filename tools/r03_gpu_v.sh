#!/bin/bash
# Round 3, GPU call V: the KC step's wall time statement by statement
# (tools/kc_gap.py), default heap and the opt-in large-block heap policy.
set -uo pipefail
O=$PWD/gpurun_out/r3v
mkdir -p $O
T() { timeout -k 10 "$@"; }
T 200 python -u tools/kc_gap.py > $O/gap_default.json 2> $O/gap_default.err || exit 11
T 200 python -u tools/kc_gap.py --heap > $O/gap_heap.json 2> $O/gap_heap.err || exit 12
