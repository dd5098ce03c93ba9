#!/bin/bash
# Counter passes for bench.py (one rocprofv3 process per pass; --pmc never
# combined with tracing).  Usage: tools/pmc_run.sh OUTDIR [bench args...]
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/$1; shift
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
# PMC_PASSES=traffic: only the two HBM-traffic passes (tools/pmc_traffic.py)
if [ "${PMC_PASSES:-all}" = "traffic" ]; then
  PASSES=("FETCH_SIZE" "WRITE_SIZE")
else
  PASSES=("FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT"
          "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU"
          "GRBM_GUI_ACTIVE SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR")
fi
for pmc in "${PASSES[@]}"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $pmc --output-format csv -d "$OUT/pass$i" -o p -- \
      python "$R/bench.py" --no-cpu-baseline --no-kernel-events "$@" > "$OUT/pass$i.log" 2>&1
done
