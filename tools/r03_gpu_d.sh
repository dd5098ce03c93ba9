#!/bin/bash
# Round 3, GPU call D: -m gpu suite (fused round-end encode, pinned vs
# pageable one-tensor calls, rowA2 without spills), round-end bench fused vs
# unfused (ResNet-50 x 4 collaborators, Llama-3-8B x 2), end-to-end loopback
# with pinned staging (default) and the pageable path, per-call overhead.
# Outputs under gpurun_out/r3d/.
set -uo pipefail
R=$PWD
O=$R/gpurun_out/r3d
mkdir -p $O
T() { timeout -k 10 "$@"; }
T 700 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest_gpu.log
[ $rc -le 1 ] || exit 13
T 300 python -u tools/roundend_bench.py --workload resnet50_fp32 --collaborators 4 --steps 50 --warmup 5 --host-steps 0 > $O/roundend_resnet50_c4.json 2> $O/roundend_resnet50.err || exit 14
T 400 python -u tools/roundend_bench.py --workload llama3_8b_fp32_update --collaborators 2 --steps 4 --warmup 1 --host-steps 0 > $O/roundend_llama_c2.json 2> $O/roundend_llama.err || exit 15
T 300 python -u tools/e2e_bench.py --out $O/e2e_pinned.json > $O/e2e_pinned.log 2>&1 || exit 16
T 300 env OFL_PLUGIN_PAGEABLE=1 python -u tools/e2e_bench.py --modes plugin --out $O/e2e_pageable.json > $O/e2e_pageable.log 2>&1 || exit 17
T 300 python -u tools/e2e_bench.py --modes plugin --out $O/e2e_pinned2.json > $O/e2e_pinned2.log 2>&1 || exit 18
T 300 python -u tools/call_overhead_probe.py > $O/call_overhead.json 2> $O/call_overhead.err || exit 19
