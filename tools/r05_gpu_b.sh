#!/bin/bash
# Round 5, GPU call b: the Eden dataflow A/B microbenchmark (tools/dataflow_bench.hip)
# and the TLZ encoder's phase times.  Outputs: gpurun_out/r05b/
set -uo pipefail
R=$PWD
O=$R/gpurun_out/r05b
mkdir -p $O
T() { timeout -k 10 "$@"; }
T 300 tools/bin/dataflow_bench 30 5 > $O/dataflow_bench.txt 2>&1; rc=$?
echo "dataflow rc=$rc" >> $O/dataflow_bench.txt
[ $rc -eq 0 ] || exit 12
OFL_GZ_PHASES=1 T 120 python -u tools/tlz_phases.py > $O/tlz_phases.txt 2>&1 || exit 13
echo "r05b done"
