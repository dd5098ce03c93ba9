#!/bin/bash
# Round 3, GPU call E: -m gpu suite (contraction-free sums of squares, the
# small-set launch, zero-copy call contexts), ResNet-50 A/B of the small-set
# launch (sset) interleaved, the Llama default line, end-to-end loopback with
# phase breakdown, per-call overhead.  Outputs under gpurun_out/r3e/.
set -uo pipefail
R=$PWD
O=$R/gpurun_out/r3e
mkdir -p $O
T() { timeout -k 10 "$@"; }
T 700 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest_gpu.log
[ $rc -le 1 ] || exit 13
for rep in 1 2 3; do
  for v in "sset" "nosset:OFL_EDEN_SSET=0" "onewave:OFL_EDEN_SPLIT_MIB=100000"; do
    n=${v%%:*}; e=""; [ "$n" != "$v" ] && e=${v#*:}
    T 200 env $e python -u bench.py --workload resnet50_fp32 --steps 400 --warmup 30 --also '' --no-cpu-baseline --no-kernel-events > $O/rn_${rep}_$n.json 2> $O/rn_${rep}_$n.err || exit 16
  done
done
T 300 python -u tools/e2e_bench.py --out $O/e2e.json > $O/e2e.log 2>&1 || exit 17
T 300 env OFL_PLUGIN_MAPPED=0 python -u tools/e2e_bench.py --modes plugin --out $O/e2e_nomap.json > $O/e2e_nomap.log 2>&1 || exit 18
T 300 python -u tools/call_overhead_probe.py > $O/call_overhead.json 2> $O/call_overhead.err || exit 19
T 600 python -u bench.py > $O/bench.json 2> $O/bench.err || exit 20
cd /tmp && export TMPDIR=/tmp
T 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/rn_trace -o k -- python3 $R/bench.py --workload resnet50_fp32 --steps 50 --warmup 10 --also '' --no-cpu-baseline --no-kernel-events > $O/rn_trace.json 2> $O/rn_trace.err || exit 21
