#!/bin/bash
# r06 end-to-end ResNet-50 loopback (BASELINE config 5): every mode the median
# of 6 rounds after a warm-up round; then the per-call overhead probe and the
# plugin phase breakdown.  Outputs: gpurun_out/r06_e2e/
set -uo pipefail
R=$PWD
O=$R/gpurun_out/r06_e2e
mkdir -p $O
timeout -k 10 400 python -u tools/e2e_bench.py --modes plugin,plugin_concurrent,batched,cpu --out $O/e2e.json > $O/e2e.log 2>&1 || exit 2
timeout -k 10 300 python -u tools/plugin_phases.py > $O/plugin_phases.json 2> $O/plugin_phases.err || exit 3
timeout -k 10 300 python -u tools/call_overhead_probe.py > $O/call_overhead.json 2> $O/call_overhead.err || exit 4
echo e2e done
