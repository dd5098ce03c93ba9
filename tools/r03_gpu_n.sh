#!/bin/bash
# Round 3, GPU call N: one-tensor host calls ending in a polled wait
# (OFL_SPIN_US=200, default) vs a blocking hipStreamSynchronize
# (OFL_SPIN_US=0): per-call overhead and the ResNet-50 loopback, alternated;
# the GPU parity suite's plugin tests.  gpurun_out/r3n/.
set -uo pipefail
R=$PWD
O=$R/gpurun_out/r3n
mkdir -p $O
T() { timeout -k 10 "$@"; }
T 400 python -u -m pytest tests/test_gpu_e2e.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || exit 11
for rep in 1 2; do
  for v in "spin" "block:OFL_SPIN_US=0"; do
    n=${v%%:*}; e=""; [ "$n" != "$v" ] && e=${v#*:}
    T 300 env $e python -u tools/call_overhead_probe.py > $O/co_${rep}_$n.json 2> $O/co_${rep}_$n.err || exit 12
    T 300 env $e python -u tools/e2e_bench.py --modes plugin --out $O/e2e_${rep}_$n.json > $O/e2e_${rep}_$n.log 2>&1 || exit 13
  done
done
