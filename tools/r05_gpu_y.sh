#!/bin/bash
# Round 5, GPU call y: host topology of the box (NUMA node of the GPU vs the allowed CPUs).
set -uo pipefail
R=$PWD
O=$R/gpurun_out/r05y
mkdir -p $O
timeout -k 10 120 python -u tools/numa_probe.py > $O/numa.json 2> $O/numa.err || exit 11
echo "r05y done"
