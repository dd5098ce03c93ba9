#!/bin/bash
# Round-4 closing evidence for the KC path on the final tree (one GPU call):
# -m gpu suite, KC 10-step line, rocprofv3 kernel stats and PMC traffic of the
# KC step, then the default bench line with that traffic.  Outputs under
# gpurun_out/kc_final/; the PMC summary also replaces the box copy of
# profiles/r04_final_kc_pipeline_hbm_traffic.json (bench.py's KC traffic source).
set -uo pipefail
R=$PWD
O=$R/gpurun_out/kc_final
mkdir -p $O
T() { timeout -k 10 "$@"; }
T 700 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest_gpu.log
[ $rc -eq 0 ] || exit 11
T 300 python -u tools/kc_bench.py --steps 10 --warmup 2 > $O/kc_bench.json 2> $O/kc_bench.err || exit 15
cd /tmp && export TMPDIR=/tmp
T 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kc_trace -o k -- python3 $R/tools/kc_bench.py --steps 3 --warmup 1 > $O/kc_trace.log 2>&1 || exit 24
T 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/kc_pmc/pass1 -o p -- python3 $R/tools/kc_bench.py --steps 3 --warmup 1 > $O/kc_pmc1.log 2>&1 || exit 25
T 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/kc_pmc/pass2 -o p -- python3 $R/tools/kc_bench.py --steps 3 --warmup 1 > $O/kc_pmc2.log 2>&1 || exit 26
cd $R && python tools/pmc_traffic.py $O/kc_pmc 4 $O/kc_traffic.json > /dev/null || exit 27
cp $O/kc_traffic.json profiles/r04_final_kc_pipeline_hbm_traffic.json
T 600 python -u bench.py > $O/bench.json 2> $O/bench.err || exit 14
echo "kc final done"
