#!/bin/bash
# Round 3, GPU call H: the exact multi-threaded seed sum (csrc/serial_sum.cpp)
# on the box's cores: its tests, its rate against the plain chain, and the
# end-to-end ResNet-50 loopback (plugin per tensor) with and without the
# opt-in heap policy; per-call overhead.  Outputs under gpurun_out/r3h/.
set -uo pipefail
R=$PWD
O=$R/gpurun_out/r3h
mkdir -p $O
T() { timeout -k 10 "$@"; }
T 300 python -u -m pytest tests/test_serial_sum.py -q > $O/pytest_sum.log 2>&1 || exit 11
T 300 python -u tools/sum_rate.py > $O/sum_rate.log 2>&1 || exit 12
T 300 python -u tools/e2e_bench.py --modes plugin,batched --out $O/e2e.json > $O/e2e.log 2>&1 || exit 13
T 300 python -u tools/e2e_bench.py --modes plugin,batched --heap-policy --out $O/e2e_heap.json > $O/e2e_heap.log 2>&1 || exit 14
T 300 python -u tools/call_overhead_probe.py > $O/call_overhead.json 2> $O/call_overhead.err || exit 15
# Llama step: two-blocks-per-CU row kernels forced on for the 2 GiB waves (A/B)
for rep in 1 2; do
  for v in "default" "row2:OFL_EDEN_ROW2=1"; do
    n=${v%%:*}; e=""; [ "$n" != "$v" ] && e=${v#*:}
    T 300 env $e python -u bench.py --steps 10 --warmup 3 --also '' --no-cpu-baseline > $O/llama_${rep}_$n.json 2> $O/llama_${rep}_$n.err || exit 16
  done
done
