#!/bin/bash
# Round 3, GPU call C: -m gpu suite, per-call overhead and end-to-end
# loopback after the pageable-source host calls, an interleaved ResNet-50 A/B
# of the schedule changes, and the round-3 evidence: PMC HBM traffic of the
# Llama bench and of the KC pipeline (tools/kc_bench.py alone), the default
# bench line with that traffic, rocprofv3 kernel stats (default and one
# stream, KC).  Outputs under gpurun_out/r3c/.
set -uo pipefail
R=$PWD
O=$R/gpurun_out/r3c
mkdir -p $O
T() { timeout -k 10 "$@"; }
T 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest_gpu.log
[ $rc -le 1 ] || exit 13
T 300 python -u tools/call_overhead_probe.py > $O/call_overhead.json 2> $O/call_overhead.err || exit 14
T 300 python -u tools/e2e_bench.py --out $O/e2e_resnet50.json > $O/e2e.log 2>&1 || exit 15
for rep in 1 2 3; do
  for v in "auto" "row2off:OFL_EDEN_ROW2=0" "small1:OFL_EDEN_SMALL2=0"; do
    n=${v%%:*}; e=""; [ "$n" != "$v" ] && e=${v#*:}
    T 200 env $e python -u bench.py --workload resnet50_fp32 --steps 400 --warmup 30 --also '' --no-cpu-baseline --no-kernel-events > $O/rn_${rep}_$n.json 2> $O/rn_${rep}_$n.err || exit 16
  done
done
PMC_PASSES=traffic T 600 bash tools/pmc_run.sh gpurun_out/r3c/pmc --steps 5 --warmup 2 --also "" || exit 17
python tools/pmc_traffic.py $O/pmc 7 $O/hbm_traffic.json > /dev/null || exit 18
T 600 python -u bench.py --traffic-json $O/hbm_traffic.json > $O/bench.json 2> $O/bench.err || exit 19
cd /tmp && export TMPDIR=/tmp
T 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/kc_pmc/pass1 -o p -- python $R/tools/kc_bench.py --steps 3 --warmup 1 > $O/kc_pmc1.log 2>&1 || exit 20
T 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/kc_pmc/pass2 -o p -- python $R/tools/kc_bench.py --steps 3 --warmup 1 > $O/kc_pmc2.log 2>&1 || exit 21
T 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kc_trace -o k -- python $R/tools/kc_bench.py --steps 3 --warmup 1 > $O/kc_trace.log 2>&1 || exit 22
T 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_default -o run -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --also "" > $O/bench_default_under_rocprof.json 2> $O/prof_default.err || exit 23
T 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_1stream -o run -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --also "" --streams 1 > $O/bench_1stream_under_rocprof.json 2> $O/prof_1stream.err || exit 24
