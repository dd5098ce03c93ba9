#!/bin/bash
# Round 3, GPU call F: -m gpu suite (early-exit small-set waves, one wave
# beside the small-set launch, pinned-staging decode + threaded copy), the
# ResNet-50 line (eager + graph) and its kernel trace, end-to-end loopback
# with phase breakdown, per-call overhead.  Outputs under gpurun_out/r3f/.
set -uo pipefail
R=$PWD
O=$R/gpurun_out/r3f
mkdir -p $O
T() { timeout -k 10 "$@"; }
T 700 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest_gpu.log
[ $rc -le 1 ] || exit 13
T 300 python -u tools/e2e_bench.py --out $O/e2e.json > $O/e2e.log 2>&1 || exit 17
T 300 python -u tools/call_overhead_probe.py > $O/call_overhead.json 2> $O/call_overhead.err || exit 19
for rep in 1 2; do
  for v in "default" "twowave:OFL_EDEN_SPLIT_MIB=0"; do
    n=${v%%:*}; e=""; [ "$n" != "$v" ] && e=${v#*:}
    T 300 env $e python -u bench.py --workload uniform_1gib --steps 5 --warmup 2 --also resnet50_fp32 --also-steps 400 --no-cpu-baseline > $O/rn_${rep}_$n.json 2> $O/rn_${rep}_$n.err || exit 16
  done
done
cd /tmp && export TMPDIR=/tmp
T 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/rn_trace -o k -- python3 $R/bench.py --workload resnet50_fp32 --steps 50 --warmup 10 --also '' --no-cpu-baseline --no-kernel-events > $O/rn_trace.json 2> $O/rn_trace.err || exit 21
