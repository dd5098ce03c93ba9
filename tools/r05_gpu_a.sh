#!/bin/bash
# Round 5, first GPU call: the -m gpu suite on the hostmem / TLZ-bounds /
# staging-ring changes, the KC line, and PMC passes of the KC step (the TLZ
# encoder's limiter: VALU / LDS / waits / occupancy).  Outputs: gpurun_out/r05a/
set -uo pipefail
R=$PWD
O=$R/gpurun_out/r05a
mkdir -p $O
T() { timeout -k 10 "$@"; }
T 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest_gpu.log
[ $rc -eq 0 ] || exit 11
T 300 python -u tools/kc_bench.py --steps 10 --warmup 2 > $O/kc_bench.json 2> $O/kc_bench.err || exit 15
cd /tmp && export TMPDIR=/tmp
T 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kc_trace -o k -- python3 $R/tools/kc_bench.py --steps 3 --warmup 1 > $O/kc_trace.log 2>&1 || exit 24
i=0
for pmc in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_ANY" \
           "GRBM_GUI_ACTIVE SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_SALU SQ_WAIT_INST_ANY"; do
  i=$((i+1))
  T 120 rocprofv3 --pmc $pmc --output-format csv -d $O/kc_sq/pass$i -o p -- python3 $R/tools/kc_bench.py --steps 2 --warmup 1 > $O/kc_sq$i.log 2>&1
  rc=$?; [ $rc -eq 0 ] || echo "pass $i rc=$rc" >> $O/pmc_fail.txt
  [ $rc -eq 124 ] || [ $rc -eq 137 ] && exit 30
done
cd $R && python tools/pmc_kernels.py $O/kc_sq $O/kc_sq.json tlz gzip > $O/kc_sq.txt 2>&1
echo "r05a done"
