#!/bin/bash
# Round-6 evidence on the final tree, one GPU call (repo root on the box):
#   bash tools/r06_evidence.sh TAG [a|b]   (a: tests, Llama PMC, bench, Llama rocprof;
#                                           b: the rest; default both -- over gpurun's 20 min)
# -m gpu suite; PMC HBM traffic of the Llama-3-8B step and the default bench
# line with it; rocprofv3 kernel stats (default and one stream) of the Llama
# step and of ResNet-50; KC pipeline: 10-step line, kernel trace, PMC passes;
# aggregator round end (fused); end-to-end ResNet-50 loopback; per-call
# overhead; seed-sum rates.  Outputs under gpurun_out/evidence_TAG/.
set -uo pipefail
TAG=${1:-r06}
R=$PWD
O=$R/gpurun_out/evidence_$TAG
mkdir -p $O
T() { timeout -k 10 "$@"; }
PART=${2:-ab}
if [[ $PART == *a* ]]; then
T 700 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest_gpu.log
[ $rc -eq 0 ] || exit 11
PMC_PASSES=traffic T 600 bash tools/pmc_run.sh gpurun_out/evidence_$TAG/pmc --steps 5 --warmup 2 --also "" || exit 12
python tools/pmc_traffic.py $O/pmc 7 $O/hbm_traffic.json > /dev/null || exit 13
T 600 python -u bench.py --traffic-json $O/hbm_traffic.json > $O/bench.json 2> $O/bench.err || exit 14
echo "bench done"
cd /tmp && export TMPDIR=/tmp
T 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_default -o run -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --also "" > $O/bench_default_under_rocprof.json 2> $O/prof_default.err || exit 21
T 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_1stream -o run -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --also "" --streams 1 > $O/bench_1stream_under_rocprof.json 2> $O/prof_1stream.err || exit 22
cd $R
echo "part a done"
fi
if [[ $PART == *b* ]]; then
T 300 python -u tools/kc_bench.py --steps 10 --warmup 2 > $O/kc_bench.json 2> $O/kc_bench.err || exit 15
T 300 python -u tools/roundend_bench.py --workload resnet50_fp32 --collaborators 4 --steps 50 --warmup 5 > $O/roundend_resnet50_c4.json 2> $O/roundend_rn.err || exit 16
T 400 python -u tools/roundend_bench.py --workload llama3_8b_fp32_update --collaborators 2 --steps 4 --warmup 1 --host-steps 0 > $O/roundend_llama_c2.json 2> $O/roundend_llama.err || exit 17
T 400 python -u tools/e2e_bench.py --modes plugin,plugin_concurrent,batched,cpu --out $O/e2e_resnet50.json > $O/e2e.log 2>&1 || exit 18
T 300 python -u tools/plugin_phases.py > $O/plugin_phases.json 2> $O/plugin_phases.err || exit 28
T 300 python -u tools/call_overhead_probe.py > $O/call_overhead.json 2> $O/call_overhead.err || exit 19
T 200 python -u tools/sum_rate.py > $O/sum_rate.log 2>&1 || exit 20
cd /tmp && export TMPDIR=/tmp
T 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_resnet -o run -- python3 $R/bench.py --workload resnet50_fp32 --steps 50 --warmup 10 --also "" --no-cpu-baseline --no-kernel-events > $O/resnet_under_rocprof.json 2> $O/prof_resnet.err || exit 23
T 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kc_trace -o k -- python3 $R/tools/kc_bench.py --steps 3 --warmup 1 > $O/kc_trace.log 2>&1 || exit 24
T 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/kc_pmc/pass1 -o p -- python3 $R/tools/kc_bench.py --steps 3 --warmup 1 > $O/kc_pmc1.log 2>&1 || exit 25
T 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/kc_pmc/pass2 -o p -- python3 $R/tools/kc_bench.py --steps 3 --warmup 1 > $O/kc_pmc2.log 2>&1 || exit 26
cd $R && python tools/pmc_traffic.py $O/kc_pmc 4 $O/kc_traffic.json > /dev/null || exit 27
# the encoder's limiter: SQ counters of the KC kernels (3 passes, <= 8 SQ each)
cd /tmp
i=0
for pmc in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_ANY" \
           "GRBM_GUI_ACTIVE SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_SALU SQ_WAIT_INST_ANY"; do
  i=$((i+1))
  T 120 rocprofv3 --pmc $pmc --output-format csv -d $O/kc_sq/pass$i -o p -- python3 $R/tools/kc_bench.py --steps 2 --warmup 1 > $O/kc_sq$i.log 2>&1 || exit $((30+i))
done
cd $R && python tools/pmc_kernels.py $O/kc_sq $O/kc_sq.json tlz gzip bkm > $O/kc_sq.txt 2>&1
echo "part b done"
fi
echo "evidence done"
