#!/bin/bash
# Round 3, GPU call B: the -m gpu suite (incl. the two-block row kernels and
# the split small-slice streams), ResNet-50 A/B of those two schedule
# changes, the default bench, and the KC pipeline's rocprofv3 evidence
# (kernel trace + FETCH_SIZE / WRITE_SIZE passes of tools/kc_bench.py alone).
set -uo pipefail
R=$PWD
O=$R/gpurun_out/r3b
mkdir -p $O
T() { timeout -k 10 "$@"; }
# test failures (rc 1) are recorded and the measurements still run; a crash,
# hang or timeout (any other rc) ends the call
T 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest_gpu.log
[ $rc -le 1 ] || exit 13
i=0
for v in "auto" "row2off:OFL_EDEN_ROW2=0" "small1:OFL_EDEN_SMALL2=0" "both_off:OFL_EDEN_ROW2=0 OFL_EDEN_SMALL2=0" "auto" "row2on:OFL_EDEN_ROW2=1"; do
  i=$((i+1)); n=${v%%:*}; e=""; [ "$n" != "$v" ] && e=${v#*:}
  T 200 env $e python -u bench.py --workload resnet50_fp32 --steps 300 --warmup 20 --also '' --no-cpu-baseline > $O/resnet_${i}_$n.json 2> $O/resnet_${i}_$n.err || exit 14
done
T 200 python -u bench.py --workload uniform_1gib --steps 50 --warmup 5 --also '' --no-cpu-baseline > $O/uniform_auto.json 2> $O/uniform_auto.err || exit 15
T 300 python -u tools/call_overhead_probe.py > $O/call_overhead.json 2> $O/call_overhead.err || exit 21
T 300 env OFL_PLUGIN_CTX=0 python -u tools/call_overhead_probe.py > $O/call_overhead_noctx.json 2> $O/call_overhead_noctx.err || exit 22
T 300 python -u tools/e2e_bench.py --out $O/e2e_resnet50.json > $O/e2e.log 2>&1 || exit 23
T 400 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err || exit 16
T 200 python -u tools/kc_bench.py --steps 10 --warmup 2 > $O/kc_pair.json 2> $O/kc_pair.err || exit 24
T 200 env OFL_GZ_PAIR=0 python -u tools/kc_bench.py --steps 10 --warmup 2 > $O/kc_nopair.json 2> $O/kc_nopair.err || exit 25
T 200 python -u tools/kc_bench.py --steps 10 --warmup 2 > $O/kc_pair2.json 2> $O/kc_pair2.err || exit 26
cd /tmp && export TMPDIR=/tmp
T 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kc_trace -o k -- python $R/tools/kc_bench.py --steps 3 --warmup 1 > $O/kc_trace.log 2>&1 || exit 17
T 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/kc_pmc/pass1 -o p -- python $R/tools/kc_bench.py --steps 3 --warmup 1 > $O/kc_pmc1.log 2>&1 || exit 18
T 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/kc_pmc/pass2 -o p -- python $R/tools/kc_bench.py --steps 3 --warmup 1 > $O/kc_pmc2.log 2>&1 || exit 19
T 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/rn_trace -o k -- python $R/bench.py --workload resnet50_fp32 --steps 100 --warmup 10 --also '' --no-cpu-baseline --no-kernel-events > $O/rn_trace.log 2>&1 || exit 20
