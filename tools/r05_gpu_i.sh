#!/bin/bash
# Round 5, GPU call i: the per-tensor plugin path -- large-call breakdown and
# the ResNet-50 loopback (default host memory, and the opt-in heap policy).
set -uo pipefail
R=$PWD
O=$R/gpurun_out/r05i
mkdir -p $O
T() { timeout -k 10 "$@"; }
T 300 python -u tools/big_call_probe.py > $O/big_call.txt 2>&1 || exit 11
T 300 python -u tools/e2e_bench.py --modes plugin,plugin_concurrent_nocombine --out $O/e2e.json > $O/e2e.log 2>&1 || exit 12
T 300 python -u tools/e2e_bench.py --modes plugin,plugin_concurrent_nocombine --heap-policy --out $O/e2e_heap.json > $O/e2e_heap.log 2>&1 || exit 13
echo "r05i done"
