#!/bin/bash
# Round 5, GPU call t: decode kernels' per-member timing (OFL_TLZ_DEC_STATS) and a stream head dump.
set -uo pipefail
R=$PWD
O=$R/gpurun_out/r05t
mkdir -p $O
T() { timeout -k 10 "$@"; }
OFL_TLZ_DEC_STATS=1 PROBE_DUMP=$O/head.gz T 300 python -u tools/kc_inflate_probe.py > $O/stats.txt 2> $O/stats.err || exit 11
echo "r05t done"
