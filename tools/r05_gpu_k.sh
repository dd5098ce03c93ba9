#!/bin/bash
# Round 5, GPU call k: the exact serial sum with multi-run phase B (and the
# AVX2 clone, 16 threads): sum phases, large-call breakdown, e2e loopback.
set -uo pipefail
R=$PWD
O=$R/gpurun_out/r05k
mkdir -p $O
T() { timeout -k 10 "$@"; }
T 300 python -u -m pytest tests/test_serial_sum.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "serial or seed or reference or pipeline" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest.log
[ $rc -eq 0 ] || exit 11
OFL_SUM_DEBUG=1 T 200 python -u tools/sum_debug_probe.py > $O/sum.txt 2>&1 || exit 12
T 300 python -u tools/big_call_probe.py > $O/big_call.txt 2>&1 || exit 13
T 300 python -u tools/e2e_bench.py --modes plugin,plugin_concurrent_nocombine --out $O/e2e.json > $O/e2e.log 2>&1 || exit 14
echo "r05k done"
